#!/bin/bash
# Focused call: a -k subset of the GPU parity suite, then one bench.py workload.
# usage: tools/gpu_quick.sh "<pytest -k expr>" "<bench.py args>"
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "$1"
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
if [ -n "$2" ]; then
  tools/gpu_step.sh quickbench 300 python -u bench.py $2
  grep -h '^{' gpurun_out/quickbench.log
fi
