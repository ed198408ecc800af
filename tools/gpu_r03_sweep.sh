#!/bin/bash
# r03 sweeps: C1 windows per launch, C3 / C1 scan blocks and windows in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sw; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-verify"
for nb in 8 16; do
  timeout -k 10 120 $B --workload range --points 1000000 --steps 200 --warmup 20 --range-batch $nb > $O/c1_b$nb.log 2>&1 || exit 1
done
for st in 2 3; do
  timeout -k 10 120 $B --workload ppoly --steps 40 --warmup 5 --range-streams $st --range-blocks 512,1024,2048 > $O/c3_s$st.log 2>&1 || exit 1
  timeout -k 10 120 $B --workload range --points 10000000 --steps 60 --warmup 10 --range-streams $st --range-blocks 512,1024,2048 > $O/c1m10_s$st.log 2>&1 || exit 1
done
# the polygon lines with their multi-thread CPU baselines
timeout -k 10 300 python -u bench.py --workload polyknn --steps 30 --warmup 5 --cpu-seconds 5 > $O/wl_polyknn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 --cpu-seconds 5 > $O/wl_pjoin.log 2>&1 || exit 1
