#!/bin/bash
# rocprofv3 PMC passes for one kernel of one bench command (each pass its own run, per the
# gfx950 slot limits: <= 8 SQ, <= 4 TCC -- FETCH_SIZE uses 3, WRITE_SIZE 2 -- so they never share).
# usage: [PASSES="fetch write lds occ"] tools/gpu_pmc.sh TAG KERNEL_REGEX bench.py-args...
# Output: gpurun_out/pmc/<TAG>/<pass>/..._counter_collection.csv (tools/pmc_summary.py reads them)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; re=$2; shift 2
O=gpurun_out/pmc/$tag
mkdir -p $O
run() {  # pass-name counters...
  local p=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$re" -d $O/$p -o $p --output-format csv \
    -- python -u bench.py "${ARGS[@]}" > $O/$p.log 2>&1 || { echo "[pmc $tag/$p] failed rc=$?"; tail -5 $O/$p.log; exit 1; }
  echo "[pmc $tag/$p] ok"
}
ARGS=("$@")
for p in ${PASSES:-fetch write lds occ}; do
  case $p in
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    lds) run lds SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES ;;
    # occupancy: mean resident waves = SQ_WAVE_CYCLES over the kernel's busy cycles (tools/pmc_table.py);
    # SQ_LEVEL_WAVES / SQ_ACCUM_PREV_HIRES read 0 on gfx950 under rocprofv3 (r02-r04 files), so not used
    occ) run occ SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT ;;
    mem) run mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAVES ;;
  esac
done
