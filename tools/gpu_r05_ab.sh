#!/bin/bash
# round 5 A/B on one box: product library vs an experiment library (GF_LIB_PATH), same command.
# usage: tools/gpu_r05_ab.sh EXPLIB "bench.py args" [EXPLIB2 ...]  (each arm runs twice, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
args=$1; shift
for rep in 1 2; do
  $S ab_base_$rep 400 python -u bench.py $args --no-cpu-baseline --no-verify || exit 1
  for v in "$@"; do
    GF_LIB_PATH=explibs/$v/libgeoflink_hip.so $S ab_${v}_$rep 400 python -u bench.py $args --no-cpu-baseline --no-verify || exit 1
  done
done
for f in gpurun_out/ab_*.log; do echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("breakdown"))')"; done
