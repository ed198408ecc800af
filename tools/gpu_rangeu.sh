#!/bin/bash
# C3 scan: pipeline depth (GF_RANGE_U) and grid size sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh ru_base 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 --no-verify --range-blocks 512,1024,1536,2048 || exit 1
for d in explibs/*/; do
  n=$(basename $d)
  GF_LIB_PATH=$d/libgeoflink_hip.so tools/gpu_step.sh ru_$n 300 python -u bench.py --workload ppoly --steps 30 --warmup 5 --no-verify --range-blocks 1024,2048 || exit 1
done
GF_LIB_PATH=explibs/GF_RANGE_U=4/libgeoflink_hip.so tools/gpu_step.sh ru4_range 300 python -u bench.py --workload range --steps 50 --warmup 5 --no-verify || exit 1
for f in gpurun_out/ru*.log; do echo $f; grep -h '^{' $f | python3 -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(" ", d["config"]["workload"], d["config"]["scan_blocks"], d["ms_per_step"], d.get("breakdown"))'; done
