#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "join_ppoly" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
tools/gpu_step.sh pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 || exit 1
GF_LIB_PATH=explibs/GF_EXP_JLANE/libgeoflink_hip.so tools/gpu_step.sh pjoin_lane 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 --no-verify || exit 1
mkdir -p gpurun_out/pj
tools/gpu_step.sh st_pjoin 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pj -o pjoin --output-format csv -- python -u bench.py --workload pjoin --steps 10 --warmup 2 --no-verify || exit 1
for f in pjoin pjoin_lane; do grep -h '^{' gpurun_out/$f.log | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["config"]["workload"], "%.3g"%d["value"], d["ms_per_step"], d.get("breakdown"), d.get("verified_vs_oracle"))'; done
