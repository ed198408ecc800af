#!/bin/bash
# depth-3 kNN: parity, the bench line (verify + cpu baseline), a gloo 2-rank rehearsal of the
# exchange path, and the rocprofv3 kernel trace of the C2 bench
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof3
mkdir -p $O
tools/gpu_step.sh d3_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pipelined or knn"
tools/gpu_step.sh d3_bench 300 python -u bench.py
tools/gpu_step.sh d3_gloo 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --points 2000000
tools/gpu_step.sh d3_stats 240 rocprofv3 --kernel-trace --stats -d $O/c2_stats -o c2 --output-format csv -- python -u bench.py --steps 200 --warmup 10 --no-verify --no-cpu-baseline
f=$(find $O -name "*kernel_trace.csv" | head -1)
python tools/trace_interval.py "$f" knn_fused 20
grep -h '^{' gpurun_out/d3_bench.log gpurun_out/d3_gloo.log gpurun_out/d3_stats.log
find $O -name "*kernel_stats.csv"
