#!/bin/bash
# K2 (bucketing by cell) + the large-k kNN sorts: parity tests, the bucket line, kernel stats
export TMPDIR=/tmp
tools/gpu_step.sh k2tests 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "bucket or large or knn_k" && \
tools/gpu_step.sh k2bench 300 python -u bench.py --workload bucket --steps 20 --warmup 3 && \
tools/gpu_step.sh k2stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k2prof -o k2 --output-format csv -- python -u bench.py --workload bucket --steps 5 --warmup 1 --no-verify --no-cpu-baseline
