#!/bin/bash
# round-5 C3: lanes per queued point in the block-end candidate tests (drain_own_queue;
# explibs/tgN = GF_RANGE_TEST_GROUP=N, the product 8), C3 line A/B on one box (--no-verify), then
# the best arm's correctness: the point-polygon GPU tests with that library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for v in base tg1 tg2 tg4; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    GF_LIB_PATH=$lib $S c3g_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
  done
done
for v in tg1 tg2 tg4; do
  GF_LIB_PATH=explibs/$v/libgeoflink_hip.so $S t_c3g_$v 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "ppoly or table_defer" || exit 1
  GF_LIB_PATH=explibs/$v/libgeoflink_hip.so $S c3g_${v}_v 300 python -u bench.py --workload ppoly --steps 100 --warmup 10 --no-cpu-baseline || exit 1
done
for f in gpurun_out/c3g_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"))')"
done
grep -h "passed\|failed" gpurun_out/t_c3g_*.log || true
