#!/bin/bash
# r04: range scan whole-tile 16-B loads, K2 bounds, join scatter LDS barriers, depth 4; tests + lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_c1 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_windows.py tests/test_gpu_polyknn.py tests/test_gpu_callers.py tests/test_gpu_clustered.py tests/test_gpu_join_density.py tests/test_gpu_knn_large.py tests/test_gpu_sharding.py tests/test_shim_native.py || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_range10m 300 python -u bench.py --workload range --points 10000000 --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_ppoly 300 python -u bench.py --workload ppoly --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_range1m 300 python -u bench.py --workload range --points 1000000 --steps 64 --warmup 16 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_polyknn4 300 python -u bench.py --workload polyknn --pipeline 4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_knn4 300 python -u bench.py --pipeline 4 --steps 30 --warmup 8 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_join 400 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline || exit 1
tools/gpu_step.sh p_join 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join -o stats --output-format csv -- python -u bench.py --workload join --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
GF_RADIX_NT=512 tools/gpu_step.sh t_bucket512 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_knn_large.py -k "bucket or knn_large" || exit 1
GF_RADIX_NT=512 tools/gpu_step.sh b_bucket512 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
GF_RADIX_NT=512 tools/gpu_step.sh p_bucket512 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket512 -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
