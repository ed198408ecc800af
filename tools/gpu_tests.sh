#!/bin/bash
# A subset of the GPU suite (TESTS, pytest node ids / files) then optional bench lines (BENCH:
# ';'-separated bench.py argument lists), each step under its own time limit.
# usage: TESTS="tests/test_gpu_comm.py ..." BENCH="--workload join --steps 20; --steps 20" tools/gpu_tests.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
if [ -n "$TESTS" ]; then
  $S t_sub 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS || exit 1
  grep -q " passed" gpurun_out/t_sub.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_sub.log || exit 1
fi
i=0
IFS=';' read -ra LINES <<< "$BENCH"
for b in "${LINES[@]}"; do
  [ -z "${b// }" ] && continue
  i=$((i + 1))
  $S b_sub$i 400 python -u bench.py $b || exit 1
done
