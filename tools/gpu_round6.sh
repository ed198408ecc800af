#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh trace50 120 python -u tools/trace_select.py
K=200 tools/gpu_step.sh trace200 120 python -u tools/trace_select.py
tools/gpu_step.sh prof_p1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p1 -o p1 --output-format csv -- python -u bench.py --steps 30 --warmup 5 --no-verify --no-cpu-baseline --pipeline 1
tools/gpu_step.sh prof_p2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p2 -o p2 --output-format csv -- python -u bench.py --steps 30 --warmup 5 --no-verify --no-cpu-baseline --pipeline 2
cat gpurun_out/trace50.log gpurun_out/trace200.log
