#!/bin/bash
# PMC comparison of the join probe kernels: explibs/OLD (two passes) vs the in-tree build
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmcj
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_FLAT SQ_INSTS_BRANCH"
CMD="python -u bench.py --workload join --steps 2 --warmup 1 --no-cpu-baseline --no-verify"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  GF_LIB_PATH=explibs/OLD/libgeoflink_hip.so timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex join_row_probe -d $O/old$i -o p --output-format csv -- $CMD > $O/old$i.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex join_row_probe -d $O/new$i -o p --output-format csv -- $CMD > $O/new$i.log 2>&1
done
find $O -name "*counter_collection.csv"
