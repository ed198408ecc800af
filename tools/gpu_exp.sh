#!/bin/bash
# Time one bench workload against each experiment build in explibs/ (and the product build).
# usage: tools/gpu_exp.sh "<bench.py args>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh exp_base 200 python -u bench.py $1 || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh exp_$n 200 python -u bench.py $1 || exit 1
done
