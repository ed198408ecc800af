#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_j 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_join_density.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py -k "join" || exit 1
grep -qE "[0-9]+ (failed|error)" gpurun_out/t_j.log && { echo "[t_j] failures: no bench on this box"; exit 1; }
tools/gpu_step.sh b_join 300 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline || exit 1
tools/gpu_step.sh p_join 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join -o stats --output-format csv -- python -u bench.py --workload join --join-streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_joinc 400 python -u bench.py --workload join --clustered --steps 5 --warmup 2 --no-cpu-baseline || exit 1
