#!/bin/bash
# r03: headline kNN scan grid sweep (depth 3), 300 windows per point, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/kb; mkdir -p $O
for rep in 1 2; do
  for b in 768 1024 1280 1536 2048; do
    timeout -k 10 120 python -u bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-verify --scan-blocks $b > $O/b${b}_$rep.log 2>&1 || exit 1
    echo "$b $rep $(grep -h '^{' $O/b${b}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['window_us'])")"
  done
done
