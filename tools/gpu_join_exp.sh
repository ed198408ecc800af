#!/bin/bash
# join probe phase costs: experiment builds (tools/build_exp.sh): np = no pair push, nw = no walk,
# ns = no walk and no band staging; hu16 = histogram loads 16 per thread, sns = scatter without the
# write-out; a name without explibs/<name> = the product library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${*:-np nw ns}; do
lib=""; [ -f explibs/$v/libgeoflink_hip.so ] && lib=explibs/$v/libgeoflink_hip.so
GF_LIB_PATH=$lib tools/gpu_step.sh p_join_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join_$v -o stats --output-format csv -- python -u bench.py --workload join --join-streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
done
