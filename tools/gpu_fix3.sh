#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh fix_tests 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "pipelined"
grep -q " passed" gpurun_out/fix_tests.log && ! grep -q "FAILED\|ERROR" gpurun_out/fix_tests.log
tools/gpu_step.sh wl_sliding 400 python -u bench.py --workload sliding --steps 20 --warmup 4 --cpu-seconds 5
grep -h '^{' gpurun_out/wl_sliding.log | cut -c1-300
