#!/bin/bash
# r03: C3 scan blocks 512 vs 1024 (three windows in flight), 300 windows per point, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3b; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 150 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline --no-verify --range-blocks 512,640,768,1024 > $O/sw_$rep.log 2>&1 || exit 1
done
grep -h '^{' $O/sw_*.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'].get('scan_blocks'), d['ms_per_step'], d['breakdown']['scan_us'])"
