#!/bin/bash
# r04: LDS accesses kept in the LDS address space (no FLAT ops) in the span-prefilter range scan
# and the join probe's flush
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_i1 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_join_density.py tests/test_gpu_clustered.py tests/test_gpu_callers.py -k "range or ppoly or join or poly or table or defer" || exit 1
tools/gpu_step.sh c3 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --no-cpu-baseline || exit 1
tools/gpu_step.sh pc3 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc3 -o stats --output-format csv -- python -u bench.py --workload ppoly --range-streams 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_join 400 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline || exit 1
tools/gpu_step.sh p_join 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join -o stats --output-format csv -- python -u bench.py --workload join --join-streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh r10m 300 python -u bench.py --workload range --points 10000000 --steps 300 --warmup 30 --no-cpu-baseline || exit 1
tools/gpu_step.sh r1m 300 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --no-cpu-baseline || exit 1
tools/gpu_step.sh pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 --no-cpu-baseline || exit 1
