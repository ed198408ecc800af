#!/bin/bash
# round-5 C1 (configs[0], 1M-point windows, 16 per batched launch) grid sweep: blocks per window
# (gf_range_plan_set_tuning; 0 = auto, n / 2048 = 488 at 1M -- 7808 blocks per 16-window launch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for b in 0 64 128 256; do
    $S c1b_${b}_$rep 200 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --range-blocks $b --no-cpu-baseline --no-verify || exit 1
  done
  $S c1b_ni_$rep 200 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --no-indices --no-cpu-baseline --no-verify || exit 1
done
$S c1b_prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c1b_prof -o stats --output-format csv -- python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --range-streams 1 --no-cpu-baseline --no-verify || exit 1
for f in gpurun_out/c1b_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("scan_blocks"))')"
done
