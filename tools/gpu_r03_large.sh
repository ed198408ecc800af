#!/bin/bash
# r03: the k > 512 queued path's tests, then the sweeps and polygon lines (tools/gpu_r03_sweep.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_knn_large.py > gpurun_out/large.log 2>&1 || { tail -30 gpurun_out/large.log; exit 1; }
tail -3 gpurun_out/large.log
bash tools/gpu_r03_sweep.sh
