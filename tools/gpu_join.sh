#!/bin/bash
# join (single pass) + range (aligned dynamic LDS): parity tests, then A/B against explibs/OLD
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh join_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "join or range or ppoly or polygon"
grep -q " passed" gpurun_out/join_tests.log && ! grep -q "FAILED\|ERROR" gpurun_out/join_tests.log
B="python -u bench.py --no-cpu-baseline --no-verify"
for r in 1 2; do
  for w in join ppoly range; do
    GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh ab_${w}_old_$r 200 $B --workload $w --steps 10 --warmup 2
    tools/gpu_step.sh ab_${w}_new_$r 200 $B --workload $w --steps 10 --warmup 2
  done
done
tools/gpu_step.sh join_stats 240 rocprofv3 --kernel-trace --stats -d gpurun_out/profj -o j --output-format csv -- python -u bench.py --workload join --steps 10 --warmup 2 --no-cpu-baseline --no-verify
for f in gpurun_out/ab_*.log; do
  echo "$f $(grep -h '^{' $f | head -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["config"]["workload"], d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
