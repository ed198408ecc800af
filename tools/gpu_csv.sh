#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh csvtests 300 python -u -m pytest tests/test_gpu_csv.py -m gpu -x -v --timeout 120 --timeout-method thread
tools/gpu_step.sh csvbench 300 python -u bench.py --workload csv --steps 20 --warmup 3 --cpu-seconds 3
grep -h '^{' gpurun_out/csvbench.log || true
