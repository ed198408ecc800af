#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sb
tools/gpu_step.sh sb_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sb/base -o j --output-format csv -- python -u bench.py --workload join --steps 6 --warmup 2 --no-verify --no-cpu-baseline || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh sb_$n 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sb/$n -o j --output-format csv -- python -u bench.py --workload join --steps 6 --warmup 2 --no-verify --no-cpu-baseline || exit 1
done
for t in gpurun_out/sb/*/; do python3 -c "
import csv
tot=0
for r in csv.DictReader(open('$t/j_kernel_stats.csv')):
    if 'orow' in r['Name'] or 'probe' in r['Name']: print('$t', r['Name'][:40], round(float(r['AverageNs'])/1000,1))
"; done
