# r03: the new GPU tests (shim, sliding range, range batch, polygon depth 2) and every join
# test on the block-chunk output, then the join A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_shim_native.py tests/test_gpu_sliding.py tests/test_gpu_polyknn.py \
  "tests/test_gpu_parity.py::test_range_run_batch" tests/test_gpu_parity.py tests/test_gpu_clustered.py -k "join or shim or sliding or polyknn or batch" \
  -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r03_new.log 2>&1 && \
bash tools/gpu_r03_joinab.sh
