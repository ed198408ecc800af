#!/bin/bash
# r04: N > 1 exchange on a side stream (two ranks on one GPU, gloo), N = 1 bench unchanged
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_l1 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_a_gpu_multirank.py || exit 1
tools/gpu_step.sh b_knn 300 python -u bench.py --steps 30 --warmup 8 --no-cpu-baseline || exit 1
