#!/bin/bash
# Range kernels: parity suite, then the C1/C3 workload lines.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
tools/gpu_step.sh ppoly 300 python -u bench.py --workload ppoly --steps 20 --warmup 3
tools/gpu_step.sh range 300 python -u bench.py --workload range --steps 100 --warmup 10
grep -h '^{' gpurun_out/ppoly.log gpurun_out/range.log
