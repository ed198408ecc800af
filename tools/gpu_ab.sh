#!/bin/bash
# A/B of two builds on one box: GF_LIB_PATH=explibs/OLD vs the in-tree library, alternating
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh ab_old_$r 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-verify
  tools/gpu_step.sh ab_new_$r 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-verify
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh abs_old_$r 200 python -u bench.py --workload sliding --steps 20 --warmup 4 --no-cpu-baseline --no-verify
  tools/gpu_step.sh abs_new_$r 200 python -u bench.py --workload sliding --steps 20 --warmup 4 --no-cpu-baseline --no-verify
done
for f in ab_old_1 ab_new_1 ab_old_2 ab_new_2 abs_old_1 abs_new_1 abs_old_2 abs_new_2; do
  echo "$f $(grep -h '^{' gpurun_out/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
