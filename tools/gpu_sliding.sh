#!/bin/bash
# sliding-window pane engine: GPU parity tests, the C5 bench line, the C2 line for regression
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest ${GPU_TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread
tools/gpu_step.sh sliding 400 python -u bench.py --workload sliding --steps 20 --warmup 4 --cpu-seconds 3 ${SLIDING_ARGS}
tools/gpu_step.sh bench 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 2 --no-verify
for f in sliding bench; do grep -h '^{' gpurun_out/$f.log || true; done
