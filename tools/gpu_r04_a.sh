#!/bin/bash
# r04: multirank (String objIDs), join density, any-k kNN, sliding, String merge; join parity; C4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_step.sh t_new 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_a_gpu_multirank.py tests/test_gpu_join_density.py tests/test_gpu_knn_large.py tests/test_gpu_sliding.py tests/test_gpu_sharding.py || exit 1
tools/gpu_step.sh t_join 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "join or knn" || exit 1
tools/gpu_step.sh b_join 400 python -u bench.py --workload join --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh b_joinc 500 python -u bench.py --workload join --clustered --steps 4 --warmup 1 --no-cpu-baseline || exit 1
