#!/bin/bash
# rocprofv3 evidence for the two kNN lines: kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes
# (each pass its own run) for the C2 bench (10M-point windows) and the C5 sliding bench
# (50M-point panes).  Summaries are copied into profiles/ by the caller.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
C2="python -u bench.py --steps 10 --warmup 4 --no-verify --no-cpu-baseline"
C5="python -u bench.py --workload sliding --steps 6 --warmup 2 --no-verify --no-cpu-baseline"
tools/gpu_step.sh c2_stats 240 rocprofv3 --kernel-trace --stats -d $O/c2_stats -o c2 --output-format csv -- $C2
tools/gpu_step.sh c2_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_fused -d $O/c2_fetch -o c2f --output-format csv -- $C2
tools/gpu_step.sh c2_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn_fused -d $O/c2_write -o c2w --output-format csv -- $C2
tools/gpu_step.sh c5_stats 300 rocprofv3 --kernel-trace --stats -d $O/c5_stats -o c5 --output-format csv -- $C5
tools/gpu_step.sh c5_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_fused -d $O/c5_fetch -o c5f --output-format csv -- $C5
tools/gpu_step.sh c5_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn_fused -d $O/c5_write -o c5w --output-format csv -- $C5
find $O -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
