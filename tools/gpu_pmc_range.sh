#!/bin/bash
# PMC pass + kernel trace over the range workloads: ARITH (pp, 10M) and TABLE (ppoly, 10M).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for wl in "ppoly" "range --points 10000000"; do
  i=$((i+1))
  tools/gpu_step.sh pmc$i 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python -u bench.py --workload $wl --steps 5 --warmup 1
  i=$((i+1))
  tools/gpu_step.sh pmc$i 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python -u bench.py --workload $wl --steps 20 --warmup 2
done
