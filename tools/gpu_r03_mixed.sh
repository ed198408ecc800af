# r03: join A/B (old library vs chunk sizes), then the shim and sliding-range GPU tests
cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_joinab.sh && \
timeout -k 10 400 python -u -m pytest tests/test_shim_native.py tests/test_gpu_sliding.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_shim.log 2>&1
