#!/bin/bash
# round-5 C3 (1000 polygons x 10M points, span prefilter) A/B: tiles per pipeline stage (U, an
# experiment build: explibs/c3u3 = -DGF_RANGE_U=3; U=4 spills 556 B/lane) x blocks (512 = 2 per
# CU, the default; 768 = 3).  The C3 kernel holds 1.5 waves/SIMD (r05 occ pass), so bytes in
# flight per wave is the lever.  Arms interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for v in base c3u3; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    for b in 512 768; do
      GF_LIB_PATH=$lib $S c3_${v}_${b}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --range-blocks $b --no-cpu-baseline --no-verify || exit 1
    done
  done
done
for f in gpurun_out/c3_*_[12].log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
