#!/bin/bash
# range active-box prefilter + range_test_kernel block count: parity, then C3 / C1 per build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "range or poly" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
tools/gpu_step.sh exp_base 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
tools/gpu_step.sh expr_base 200 python -u bench.py --workload range --steps 100 --warmup 10 || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh exp_$n 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
done
GF_LIB_PATH=explibs/GF_NO_BOX/libgeoflink_hip.so tools/gpu_step.sh expr_nobox 200 python -u bench.py --workload range --steps 100 --warmup 10 || exit 1
for f in gpurun_out/exp_*.log gpurun_out/expr_*.log; do
  echo "$f"; grep -h '^{' $f | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" ", d["config"]["workload"], d["ms_per_step"], d["breakdown"], d["verified_vs_oracle"])'
done
