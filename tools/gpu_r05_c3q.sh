#!/bin/bash
# round-5 C3 experiment (not kept; the variant is not in the product): the block's candidate
# queue in LDS (its first 256 entries; a build with GF_RANGE_BLOCKQ=256, run as "base" here) vs in
# global memory (explibs/nbq, = the product).  Result: 47.8 vs 42.5 us per window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_c3q 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py tests/test_gpu_sliding.py tests/test_gpu_host_windows.py \
  -k "range or ppoly" || exit 1
grep -q " passed" gpurun_out/t_c3q.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_c3q.log || exit 1
$S c3q_v 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --cpu-seconds 2 || exit 1
for rep in 1 2; do
  for v in base nbq; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    GF_LIB_PATH=$lib $S c3q_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
  done
done
for f in gpurun_out/c3q_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"))')"
done
