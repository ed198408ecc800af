#!/bin/bash
# First-contact GPU session: smoke, parity tests, short bench, rocprof kernel trace.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh smoke 420 python -u -c "import __graft_entry__ as g; g.smoke()"
tools/gpu_step.sh gputests 700 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
tools/gpu_step.sh bench 300 python -u bench.py --steps 30 --warmup 5
