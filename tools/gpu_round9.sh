#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh bench 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 3
tools/gpu_step.sh range 300 python -u bench.py --workload range --steps 100 --warmup 10
tools/gpu_step.sh range05 300 python -u bench.py --workload range --radius 0.05 --steps 100 --warmup 10
tools/gpu_step.sh ppoly 300 python -u bench.py --workload ppoly --steps 20 --warmup 3
tools/gpu_step.sh join 300 python -u bench.py --workload join --steps 10 --warmup 2
tools/gpu_step.sh prof_wl 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wl -o wl --output-format csv -- python -u bench.py --workload range --steps 30 --warmup 5
tools/gpu_step.sh prof_wl2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wl2 -o wl2 --output-format csv -- python -u bench.py --workload join --steps 5 --warmup 1
for f in bench range range05 ppoly join; do grep -h '^{' gpurun_out/$f.log || true; done
