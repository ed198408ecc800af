#!/bin/bash
# select general path: kNN parity tests (all kNN flavours), then polygon-kNN A/B vs explibs/OLD
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh sel_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_polyknn.py tests/test_gpu_sliding.py -k "knn or poly or sliding"
grep -q " passed" gpurun_out/sel_tests.log && ! grep -q "FAILED\|ERROR" gpurun_out/sel_tests.log
B="python -u bench.py --no-cpu-baseline --workload polyknn --steps 20 --warmup 4"
for r in 1 2; do
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so tools/gpu_step.sh sel_old_$r 200 $B --no-verify
  tools/gpu_step.sh sel_new_$r 200 $B
done
for f in gpurun_out/sel_*_?.log; do
  echo "$f $(grep -h '^{' $f | head -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["breakdown"], d.get("verified_vs_oracle"))')"
done
