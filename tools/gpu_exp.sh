#!/bin/bash
# Time one bench workload against each experiment build in explibs/ (and the product build).
# usage: tools/gpu_exp.sh "<bench.py args>" [pytest -k expr run first on the product build]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
if [ -n "$2" ]; then
  tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "$2" || exit 1
  grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
fi
tools/gpu_step.sh exp_base 200 python -u bench.py $1 || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh exp_$n 200 python -u bench.py $1 || exit 1
done
