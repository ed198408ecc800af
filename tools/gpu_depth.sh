#!/bin/bash
# kNN pipeline depth 3 (two streams) vs depth 2: parity test, then alternating bench runs
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pipelined" > gpurun_out/depth_test.log 2>&1
tail -2 gpurun_out/depth_test.log
for r in 1 2; do
  for d in 2 3; do
    timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-verify --pipeline $d > gpurun_out/depth_${d}_$r.log 2>&1
    echo "depth $d run $r: $(grep -h '^{' gpurun_out/depth_${d}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"], d["breakdown"]["window_us"])')"
  done
done
