#!/bin/bash
# r04: K2 row mode (vs GF_K2_LSD=1), bounds v3 + 512-thread scatter default (+ 6-wave A/B), range 8-B loads restored, join streams A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_d1 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_knn_large.py tests/test_gpu_sharding.py -k "bucket or range or knn_large or shard" || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
GF_K2_LSD=1 tools/gpu_step.sh b_bucket_lsd 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
GF_RADIX_OCC6=1 tools/gpu_step.sh b_bucket6 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
GF_RADIX_OCC6=1 tools/gpu_step.sh p_bucket6 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket6 -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_range10m 300 python -u bench.py --workload range --points 10000000 --steps 40 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_range1m 300 python -u bench.py --workload range --points 1000000 --steps 64 --warmup 16 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_join1 400 python -u bench.py --workload join --join-streams 1 --steps 20 --warmup 3 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_join2 400 python -u bench.py --workload join --join-streams 2 --steps 20 --warmup 3 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_join3 400 python -u bench.py --workload join --join-streams 3 --steps 20 --warmup 3 --no-cpu-baseline --no-verify || exit 1
