#!/bin/bash
# r04: multirank (String objIDs), join density, any-k kNN, sliding, String merge; parity; K2 + C4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_new 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_a_gpu_multirank.py tests/test_gpu_join_density.py tests/test_gpu_knn_large.py tests/test_gpu_sliding.py tests/test_gpu_sharding.py tests/test_gpu_host_windows.py tests/test_gpu_polyknn.py || exit 1
tools/gpu_step.sh t_par 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "join or knn or bucket" || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_join 400 python -u bench.py --workload join --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh b_joinc 500 python -u bench.py --workload join --clustered --steps 4 --warmup 1 --no-cpu-baseline || exit 1
