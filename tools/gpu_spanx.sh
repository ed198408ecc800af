#!/bin/bash
# span x-cut in the range scan: whole GPU suite, then C3 / C1 lines (1 and 2 streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
tools/gpu_step.sh sx_ppoly_r1 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 --no-cpu-baseline --range-streams 1 || exit 1
tools/gpu_step.sh sx_ppoly 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
tools/gpu_step.sh sx_range 200 python -u bench.py --workload range --steps 100 --warmup 10 || exit 1
tools/gpu_step.sh sx_pjoin 200 python -u bench.py --workload pjoin --steps 20 --warmup 3 || exit 1
