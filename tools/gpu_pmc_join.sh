#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcj
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "join"
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
tools/gpu_step.sh jb 200 python -u bench.py --workload join --steps 10 --warmup 2
tools/gpu_step.sh jp1 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcj/p1 -o p1 --output-format csv -- python -u bench.py --workload join --steps 3 --warmup 1
tools/gpu_step.sh jp2 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcj/p2 -o p2 --output-format csv -- python -u bench.py --workload join --steps 5 --warmup 1
