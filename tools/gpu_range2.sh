#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "range"
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
tools/gpu_step.sh b1 300 python -u bench.py --workload ppoly --steps 20 --warmup 3 --range-blocks 0,1024,512
tools/gpu_step.sh b2 300 python -u bench.py --workload range --steps 50 --warmup 5 --range-blocks 0,1024,512
