#!/bin/bash
# r03 band probe: every join parity test, then the uniform / clustered C4 lines, kernel stats of
# the uniform line, and (EXPLIBS) the uniform line on experiment builds of the library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/band; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py \
  -m gpu -k "join" -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/tests.log; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
J="python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $J > $O/join_u.log 2>&1 && \
timeout -k 10 300 python bench.py --workload join --steps 5 --warmup 2 --no-cpu-baseline --clustered > $O/join_c.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o join --output-format csv -- python -u bench.py --workload join --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $O/join_prof.log 2>&1 || exit 1
for L in ${EXPLIBS:-}; do
  GF_LIB_PATH=explibs/$L.so timeout -k 10 200 $J --no-verify > $O/exp_$L.log 2>&1 || exit 1
done
