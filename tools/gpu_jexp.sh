#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --workload join --steps 6 --warmup 2 --no-cpu-baseline --no-verify"
for v in OLD GF_EXP_J2 GF_EXP_J1; do
  GF_LIB_PATH=explibs/$v/libgeoflink_hip.so tools/gpu_step.sh jexp_$v 200 $B || true
done
tools/gpu_step.sh jexp_new 200 $B
for f in gpurun_out/jexp_*.log; do
  echo "$f $(grep -h '^{' $f | head -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
