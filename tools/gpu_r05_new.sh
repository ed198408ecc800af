#!/bin/bash
# round 5: the new / changed GPU tests, then the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tools/gpu_step.sh t_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_comm.py tests/test_gpu_knn_ties.py} || exit 1
grep -q " passed" gpurun_out/t_new.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_new.log || exit 1
tools/gpu_step.sh b_knn 200 python -u bench.py --steps 20 --warmup 5
