#!/bin/bash
# C3 / range table-mode validation: parity tests of the range paths, the ppoly line, kernel stats
export TMPDIR=/tmp
tools/gpu_step.sh c3tests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "range or ppoly or sharding" && \
tools/gpu_step.sh c3bench 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 && \
tools/gpu_step.sh c3bench1 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 --range-streams 1 && \
tools/gpu_step.sh c3stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o c3 --output-format csv -- python -u bench.py --workload ppoly --steps 10 --warmup 2 --no-verify --no-cpu-baseline --range-streams 1
