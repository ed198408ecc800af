#!/bin/bash
# r04: span-prefilter rounds without global memory (queue classified before a queued point's tile
# leaves the ring; LDS-only span table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_k1 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_callers.py tests/test_gpu_sharding.py -k "range or ppoly or poly or table or defer or span" || exit 1
tools/gpu_step.sh c3 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline || exit 1
tools/gpu_step.sh pc3 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc3 -o stats --output-format csv -- python -u bench.py --workload ppoly --range-streams 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh c3c 300 python -u bench.py --workload ppoly --clustered --steps 100 --warmup 10 --no-cpu-baseline || exit 1
