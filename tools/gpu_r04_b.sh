#!/bin/bash
# r04: K2 (LDS-only barriers, vector bounds), range scan 16-B loads, polygon kNN depth 3, host 16 B/pt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_b1 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_a_gpu_multirank.py -k string tests/test_gpu_host_windows.py tests/test_gpu_polyknn.py tests/test_gpu_callers.py tests/test_gpu_clustered.py || exit 1
tools/gpu_step.sh t_b2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "range or ppoly or bucket or bitmap or batch" tests/test_gpu_sliding.py tests/test_gpu_sharding.py || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_range10m 300 python -u bench.py --workload range --points 10000000 --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_ppoly 300 python -u bench.py --workload ppoly --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_range1m 300 python -u bench.py --workload range --points 1000000 --steps 64 --warmup 16 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_polyknn 300 python -u bench.py --workload polyknn --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_knn 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 6 || exit 1
