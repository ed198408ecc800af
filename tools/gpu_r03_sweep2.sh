#!/bin/bash
# r03 sweeps: windows in flight for C4 (join streams 2 / 3) and C1 / C3 (range streams 3 / 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sw2; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-verify"
for st in 2 3 4; do
  timeout -k 10 200 $B --workload join --steps 24 --warmup 6 --join-streams $st > $O/join_s$st.log 2>&1 || exit 1
done
for st in 3 4; do
  timeout -k 10 120 $B --workload ppoly --steps 40 --warmup 8 --range-streams $st > $O/c3_s$st.log 2>&1 || exit 1
  timeout -k 10 120 $B --workload range --points 10000000 --steps 60 --warmup 12 --range-streams $st > $O/c1m10_s$st.log 2>&1 || exit 1
done
grep -H '^{' $O/*.log | python -c "
import json,sys
for l in sys.stdin:
    f,_,j=l.partition(':'); d=json.loads(j); print(f.split('/')[-1], d['ms_per_step'], d['value'])"
