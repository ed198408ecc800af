#!/bin/bash
# polygon-query kNN: parity tests + the line at depths 3 / 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_pk 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_polyknn.py tests/test_gpu_parity.py tests/test_gpu_callers.py tests/test_gpu_sliding.py -k "poly or ppoly_knn or knn_poly or sliding" || exit 1
tools/gpu_step.sh b_pk4 300 python -u bench.py --workload polyknn --pipeline 4 --steps 200 --warmup 10 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_pk3 300 python -u bench.py --workload polyknn --pipeline 3 --steps 200 --warmup 10 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_pk2 300 python -u bench.py --workload polyknn --pipeline 2 --steps 200 --warmup 10 --no-cpu-baseline || exit 1
tools/gpu_step.sh p_pk 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_pk -o stats --output-format csv -- python -u bench.py --workload polyknn --steps 20 --warmup 5 --no-cpu-baseline --no-verify || exit 1
