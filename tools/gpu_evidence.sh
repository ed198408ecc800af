#!/bin/bash
# round validation, part 2: the default bench line, the C2 depth-3 kernel trace (launch interval,
# tools/trace_interval.py) and every workload line (tools/gpu_workloads.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh default_bench 400 python -u bench.py || exit 1
tools/gpu_step.sh knn_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/knn_trace -o trace --output-format csv -- python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-verify || exit 1
python tools/trace_interval.py gpurun_out/knn_trace/trace_kernel_trace.csv knn_fused 10 > gpurun_out/knn_interval.txt 2>&1
cat gpurun_out/knn_interval.txt
bash tools/gpu_workloads.sh
