#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in range ppoly join pjoin; do
  tools/gpu_step.sh cb_$w 400 python -u bench.py --workload $w --steps 20 --warmup 3 || exit 1
done
for w in range ppoly join pjoin; do grep -h '^{' gpurun_out/cb_$w.log | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["config"]["workload"], "%.3g"%d["value"], d["ms_per_step"], d.get("verified_vs_oracle"), d.get("cpu_baseline",{}).get("value"))'; done
