#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for s in 1 2 3; do
  tools/gpu_step.sh rs_range_$s 300 python -u bench.py --workload range --steps 200 --warmup 20 --range-streams $s --no-cpu-baseline || exit 1
  tools/gpu_step.sh rs_ppoly_$s 300 python -u bench.py --workload ppoly --steps 40 --warmup 5 --range-streams $s --no-cpu-baseline || exit 1
done
for f in gpurun_out/rs_*.log; do echo $f; grep -h '^{' $f | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" ", d["config"]["workload"], d["config"]["windows_in_flight"], d["ms_per_step"], d["breakdown"], d["verified_vs_oracle"])'; done
