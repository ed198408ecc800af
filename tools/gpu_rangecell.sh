#!/bin/bash
# division-free cells without LDS thresholds (product) vs GF_EXP_THRESH: parity, C3/C1 timing, PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "range or poly" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
for r in 1 2; do
tools/gpu_step.sh rc_new_$r 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
GF_LIB_PATH=explibs/GF_EXP_THRESH/libgeoflink_hip.so tools/gpu_step.sh rc_old_$r 200 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
done
tools/gpu_step.sh rcr_new 200 python -u bench.py --workload range --steps 100 --warmup 10 || exit 1
mkdir -p gpurun_out/pmcr
tools/gpu_step.sh pmc_new 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY -d gpurun_out/pmcr/new -o new --output-format csv -- python -u bench.py --workload ppoly --steps 5 --warmup 1 --no-verify || exit 1
GF_LIB_PATH=explibs/GF_EXP_THRESH/libgeoflink_hip.so tools/gpu_step.sh pmc_old 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY -d gpurun_out/pmcr/old -o old --output-format csv -- python -u bench.py --workload ppoly --steps 5 --warmup 1 --no-verify || exit 1
for f in gpurun_out/rc*_*.log; do
  echo "$f"; grep -h '^{' $f | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" ", d["config"]["workload"], d["ms_per_step"], d["breakdown"], d["verified_vs_oracle"])'
done
