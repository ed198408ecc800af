#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in 256 512 768 1024 1280 2048 1024; do
  timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-verify --scan-blocks $b > gpurun_out/blk_$b.log 2>&1
  echo "$b $(grep -h '^{' gpurun_out/blk_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
