#!/bin/bash
# r04: K2 loads unconditional (clamped): hist, seg hist and scatter tiles issue all loads together
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_g1 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_knn_large.py tests/test_gpu_sharding.py -k "bucket or knn_large or shard" || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
GF_K2_LSD=1 tools/gpu_step.sh b_bucket_lsd 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
