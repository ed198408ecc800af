#!/bin/bash
# join probe phase costs: experiment builds (tools/build_exp.sh): np = no pair push, nw = no walk,
# ns = no walk and no band staging
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${*:-np nw ns}; do
GF_LIB_PATH=explibs/$v/libgeoflink_hip.so tools/gpu_step.sh p_join_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join_$v -o stats --output-format csv -- python -u bench.py --workload join --join-streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
done
