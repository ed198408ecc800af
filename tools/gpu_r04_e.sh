#!/bin/bash
# r04: K2 scatter phase costs (experiment builds: no stores / fake ranks / no LDS permutation) + PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in base rx1 rx2 rx3; do
  lib=""; [ $v != base ] && lib=explibs/$v/libgeoflink_hip.so
  GF_LIB_PATH=$lib tools/gpu_step.sh px_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/px_$v -o stats --output-format csv -- python -u bench.py --workload bucket --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
done
PASSES="lds mem occ" tools/gpu_pmc.sh r04_bucketx "radix_scatter" --workload bucket --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
