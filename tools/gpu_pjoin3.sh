#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "poly or range" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
tools/gpu_step.sh pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh ppoly 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 || exit 1
tools/gpu_step.sh polyknn 300 python -u bench.py --workload polyknn --steps 30 --warmup 5 || exit 1
mkdir -p gpurun_out/pj
tools/gpu_step.sh st_pjoin 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pj -o pjoin --output-format csv -- python -u bench.py --workload pjoin --steps 10 --warmup 2 --no-verify || exit 1
for f in pjoin ppoly polyknn; do grep -h '^{' gpurun_out/$f.log | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["config"]["workload"], "%.3g"%d["value"], d["ms_per_step"], d.get("breakdown"), d.get("verified_vs_oracle"))'; done
