#!/bin/bash
# round-5 C3 cost split (experiment builds, results wrong on purpose: --no-verify):
#   c3e1 = GF_RANGE_EXP=1: the span queue filled, no classification rounds (nothing accepted);
#   c3e3 = GF_RANGE_EXP=3: rounds, no candidate tests at the block's end;
#   c3e4 = GF_RANGE_EXP=4: rounds, the candidate points neither queued nor tested.
# (GF_RANGE_EXP=2, nothing queued, lets the compiler drop the loads: not a measurement.)
# Three windows in flight (the bench line) and one stream (per-launch kernel time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for v in base c3e1 c3e3 c3e4; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    GF_LIB_PATH=$lib $S c3s_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
    GF_LIB_PATH=$lib $S c3s1_${v}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --range-streams 1 --no-cpu-baseline --no-verify || exit 1
  done
done
for f in gpurun_out/c3s_*_[12].log gpurun_out/c3s1_*_[12].log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
