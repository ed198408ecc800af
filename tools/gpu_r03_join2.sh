#!/bin/bash
# r03 join: the band-probe global-window test + every join test, then the C4 lines with two
# windows in flight (default) and one, uniform and clustered
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/j2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py \
  -m gpu -k "join" -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/tests.log; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
J="python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $J > $O/u2.log 2>&1 && \
timeout -k 10 200 $J --join-streams 1 --no-verify > $O/u1.log 2>&1 && \
timeout -k 10 300 python bench.py --workload join --steps 5 --warmup 2 --no-cpu-baseline --clustered > $O/c2.log 2>&1 && \
timeout -k 10 300 python bench.py --workload join --steps 5 --warmup 2 --no-cpu-baseline --clustered --join-streams 1 --no-verify > $O/c1.log 2>&1
