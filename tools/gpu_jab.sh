#!/bin/bash
# join probe A/B: explibs/OLD (two passes) vs in-tree, plus the join parity tests
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh jab_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "join"
grep -q " passed" gpurun_out/jab_tests.log && ! grep -q "FAILED\|ERROR" gpurun_out/jab_tests.log
B="python -u bench.py --workload join --steps 10 --warmup 2 --no-cpu-baseline --no-verify"
for r in 1 2; do
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh jab_old_$r 200 $B
  tools/gpu_step.sh jab_new_$r 200 $B
done
tools/gpu_step.sh jab_stats 240 rocprofv3 --kernel-trace --stats -d gpurun_out/profj -o j --output-format csv -- $B
for f in gpurun_out/jab_*_?.log; do
  echo "$f $(grep -h '^{' $f | head -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
cut -d, -f1-4 gpurun_out/profj/j_kernel_stats.csv | head -8
