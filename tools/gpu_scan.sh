#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh knntests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sliding.py -m gpu -x -q --timeout 120 --timeout-method thread -k "knn or sliding"
tools/gpu_step.sh tune 300 python -u tools/tune_knn.py
tools/gpu_step.sh bench 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 2 --no-verify
tools/gpu_step.sh sliding 300 python -u bench.py --workload sliding --steps 20 --warmup 4 --no-cpu-baseline --no-verify
grep -h '^{' gpurun_out/bench.log gpurun_out/sliding.log | cut -c1-200 || true
