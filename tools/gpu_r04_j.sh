#!/bin/bash
# r04: C3 scan grid sweep after the FLAT fixes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh c3sweep 300 python -u bench.py --workload ppoly --range-blocks 256,512,768,1024,1536 --steps 300 --warmup 30 --no-cpu-baseline --no-verify || exit 1
