#!/bin/bash
# round-5 C3 blocks sweep with the two-lane drain (--range-blocks; 512 = 2 per CU, the default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for rep in 1 2; do
  for b in 384 448 512 576 640; do
    $S c3s_b${b}_$rep 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --range-blocks $b --no-cpu-baseline --no-verify || exit 1
  done
done
for f in gpurun_out/c3s_b*_[12].log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
