#!/bin/bash
# r03: range parity on the final scan, then the C3 / C1 10M workload lines and C3's PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sliding.py -k "range or ppoly" > gpurun_out/c3l_tests.log 2>&1 || { tail -30 gpurun_out/c3l_tests.log; exit 1; }
tail -2 gpurun_out/c3l_tests.log
bash tools/gpu_step.sh wl_ppoly 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --cpu-seconds 5
bash tools/gpu_step.sh wl_range10m 300 python -u bench.py --workload range --points 10000000 --steps 300 --warmup 30 --cpu-seconds 5
bash tools/gpu_pmc_r03.sh ppoly
