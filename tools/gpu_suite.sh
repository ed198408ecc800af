#!/bin/bash
# round validation, part 1: smoke and the whole GPU suite (gpurun_out/gputests.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh smoke 420 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
tools/gpu_step.sh gputests 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
