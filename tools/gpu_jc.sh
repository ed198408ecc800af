#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "join" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
mkdir -p gpurun_out/jc
tools/gpu_step.sh jc_new 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jc/new -o j --output-format csv -- python -u bench.py --workload join --steps 6 --warmup 2 --no-verify --no-cpu-baseline || exit 1
GF_LIB_PATH=explibs/GF_EXP_JC1/libgeoflink_hip.so tools/gpu_step.sh jc_old 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jc/old -o j --output-format csv -- python -u bench.py --workload join --steps 6 --warmup 2 --no-verify --no-cpu-baseline || exit 1
for t in new old; do python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/jc/$t/j_kernel_stats.csv')):
    if 'compact' in r['Name'] or 'probe' in r['Name']: print('$t', r['Name'][:40], round(float(r['AverageNs'])/1000,1))"; done
