#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
tools/gpu_step.sh tune 300 python -u tools/tune_knn.py
tools/gpu_step.sh bench 300 python -u bench.py --steps 30 --warmup 5 --cpu-seconds 3
