#!/bin/bash
# single-pass join: parity tests, then A/B against explibs/OLD (the two-pass probe)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh join_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "join"
grep -q " passed" gpurun_out/join_tests.log && ! grep -q "FAILED\|ERROR" gpurun_out/join_tests.log
for r in 1 2; do
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh joinab_old_$r 200 python -u bench.py --workload join --steps 10 --warmup 2 --no-cpu-baseline --no-verify
  tools/gpu_step.sh joinab_new_$r 200 python -u bench.py --workload join --steps 10 --warmup 2 --no-cpu-baseline --no-verify
done
tools/gpu_step.sh join_stats 240 rocprofv3 --kernel-trace --stats -d gpurun_out/profj -o j --output-format csv -- python -u bench.py --workload join --steps 10 --warmup 2 --no-cpu-baseline --no-verify
for f in joinab_old_1 joinab_new_1 joinab_old_2 joinab_new_2; do
  echo "$f $(grep -h '^{' gpurun_out/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
