#!/bin/bash
# round-5 C3 experiment (not kept; the variant is not in the product): candidate-cell points
# tested in-stream by their own wave (a build with GF_RANGE_WTEST=1) against the product's
# block-end tests (explibs/now).  The range / point-polygon GPU tests, the C3 line (verified),
# and an A/B on one box.  Result: in-stream 57.9 us vs 45.7 us per window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_rng 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py tests/test_gpu_sliding.py tests/test_gpu_host_windows.py \
  -k "range or ppoly or join_ppoly" || exit 1
grep -q " passed" gpurun_out/t_rng.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_rng.log || exit 1
$S c3w_v 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --cpu-seconds 2 || exit 1
for rep in 1 2; do
  for v in base now; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    GF_LIB_PATH=$lib $S c3w_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
    GF_LIB_PATH=$lib $S c3w1_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --range-streams 1 --no-cpu-baseline --no-verify || exit 1
  done
  for b in 768; do
    $S c3w_b${b}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --range-blocks $b --no-cpu-baseline --no-verify || exit 1
  done
done
for f in gpurun_out/c3w_v.log gpurun_out/c3w*_[12].log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"))')"
done
