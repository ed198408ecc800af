#!/bin/bash
# round-5 C1 (configs[0], 1M-point windows, 16 per batched launch) grid sweep: blocks per window
# (gf_range_plan_set_tuning; 0 = auto).  r05 first sweep (auto was n / 2048 = 488 per window,
# 7808 blocks per launch): 488 3.7-3.8 us per window, 256 3.4, 128 3.3, 64 3.2-3.3, no index
# list 3.1 -> auto now holds the launch to ~4 blocks per CU (64 per window at 16 windows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for b in 0 32 48 96; do
    $S c1b_${b}_$rep 200 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --range-blocks $b --no-cpu-baseline --no-verify || exit 1
  done
done
$S c1b_10m 200 python -u bench.py --workload range --points 10000000 --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
for f in gpurun_out/c1b_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("scan_blocks"))')"
done
