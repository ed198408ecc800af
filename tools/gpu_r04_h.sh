#!/bin/bash
# r04: C3 phase costs (experiment builds: no classification rounds / nothing queued)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in base re1 re2; do
  lib=""; [ $v != base ] && lib=explibs/$v/libgeoflink_hip.so
  GF_LIB_PATH=$lib tools/gpu_step.sh c3_$v 200 python -u bench.py --workload ppoly --steps 100 --warmup 10 --no-cpu-baseline --no-verify || exit 1
  GF_LIB_PATH=$lib tools/gpu_step.sh pc3_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc3_$v -o stats --output-format csv -- python -u bench.py --workload ppoly --range-streams 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify || exit 1
done
