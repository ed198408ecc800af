#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh pj_base 200 python -u bench.py --workload pjoin --steps 20 --warmup 3 --no-verify || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh pj_$n 200 python -u bench.py --workload pjoin --steps 20 --warmup 3 --no-verify || exit 1
done
mkdir -p gpurun_out/pjp
tools/gpu_step.sh pmc_pj 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pjp -o pjp --output-format csv -- python -u bench.py --workload pjoin --steps 3 --warmup 1 --no-verify || exit 1
for f in gpurun_out/pj_*.log; do echo $f; grep -h '^{' $f | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" ", d["ms_per_step"], d.get("breakdown"))'; done
