#!/bin/bash
# r03: C3 after the wave-queue change -- blocks x windows-in-flight sweep, then the workload line
# (with CPU baselines) and its kernel stats + PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3f; mkdir -p $O
for st in 2 3; do
  timeout -k 10 150 python -u bench.py --workload ppoly --steps 60 --warmup 9 --no-cpu-baseline --no-verify --range-streams $st --range-blocks 512,768,1024 > $O/sw_s$st.log 2>&1 || exit 1
done
grep -h '^{' $O/sw_s*.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'].get('range_streams', d['config'].get('windows_in_flight')), d['config'].get('scan_blocks'), d['ms_per_step'])"
bash tools/gpu_step.sh wl_ppoly 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 --cpu-seconds 5
bash tools/gpu_pmc_r03.sh ppoly
