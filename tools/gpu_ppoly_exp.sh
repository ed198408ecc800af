#!/bin/bash
# C3 point-polygon range scan: experiment builds (explibs/) vs the product build, one stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
A="--workload ppoly --steps 30 --warmup 5 --no-verify --no-cpu-baseline --range-streams 1"
tools/gpu_step.sh exp_base 200 python -u bench.py $A || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh exp_$n 200 python -u bench.py $A || exit 1
done
tools/gpu_step.sh exp_inline 200 python -u bench.py $A --range-defer 1 || exit 1
