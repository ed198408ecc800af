#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
tools/gpu_step.sh tune 300 python -u tools/tune_knn.py
tools/gpu_step.sh bench 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 3
tools/gpu_step.sh prof_knn 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_knn -o knn --output-format csv -- python -u bench.py --steps 30 --warmup 5 --no-verify --no-cpu-baseline
find gpurun_out/prof_knn -name "*stats*" | head
