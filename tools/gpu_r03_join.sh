# r03 join rework: parity of every join path (row fine / coarse / stream experiment, legacy,
# clustered, async, capacity, sharding) + the N>1 bench paths, then the C4 bench lines:
# uniform and clustered, default path and the streaming experiment.
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_a_gpu_multirank.py tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py -m gpu -v -k "join or two_ranks" --timeout 400 --timeout-method thread > gpurun_out/r03_join_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/r03_join_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_join_u.log 2>&1 && \
timeout -k 10 200 python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline --join-stream > gpurun_out/r03_join_us.log 2>&1 && \
timeout -k 10 300 python bench.py --workload join --steps 5 --warmup 2 --no-cpu-baseline --clustered > gpurun_out/r03_join_c.log 2>&1
