#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmccsv
B="python -u bench.py --workload csv --steps 3 --warmup 1 --no-cpu-baseline"
tools/gpu_step.sh cp1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --kernel-include-regex csv -d gpurun_out/pmccsv/p1 -o p1 --output-format csv -- $B
tools/gpu_step.sh cp2 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmccsv/p2 -o p2 --output-format csv -- $B
