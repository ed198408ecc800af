#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh wl_range 300 python -u bench.py --workload range --steps 200 --warmup 20 || exit 1
tools/gpu_step.sh wl_ppoly 300 python -u bench.py --workload ppoly --steps 40 --warmup 5 || exit 1
mkdir -p gpurun_out/wl2
for w in range ppoly; do
  tools/gpu_step.sh st2_$w 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wl2/$w -o $w --output-format csv -- python -u bench.py --workload $w --steps 20 --warmup 2 --no-verify --no-cpu-baseline || exit 1
done
grep -h '^{' gpurun_out/wl_range.log gpurun_out/wl_ppoly.log > gpurun_out/wl2/lines.jsonl
