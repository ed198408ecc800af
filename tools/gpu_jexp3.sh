#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
GF_LIB_PATH=explibs/GF_EXP_J4/libgeoflink_hip.so tools/gpu_step.sh pj_J4 200 python -u bench.py --workload pjoin --steps 2 --warmup 1 --no-verify || exit 1
GF_LIB_PATH=explibs/GF_EXP_J3/libgeoflink_hip.so tools/gpu_step.sh pj_J3 200 python -u bench.py --workload pjoin --steps 20 --warmup 3 --no-verify || exit 1
mkdir -p gpurun_out/pjp2
tools/gpu_step.sh pmc_pj 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pjp2 -o pjp --output-format csv -- python -u bench.py --workload pjoin --steps 3 --warmup 1 --no-verify || exit 1
grep -h "block" gpurun_out/pj_J4.log | head -12
grep -h '^{' gpurun_out/pj_J3.log | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" J3", d["ms_per_step"], d.get("breakdown"))'
