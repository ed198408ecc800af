#!/bin/bash
# clustered C4: probe phase costs (experiment builds np / nw)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${*:-base np nw}; do
  lib=""; [ -f explibs/$v/libgeoflink_hip.so ] && lib=explibs/$v/libgeoflink_hip.so
  GF_LIB_PATH=$lib tools/gpu_step.sh pjc_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pjc_$v -o stats --output-format csv -- python -u bench.py --workload join --clustered --join-streams 1 --steps 3 --warmup 1 --no-cpu-baseline --no-verify || exit 1
done
