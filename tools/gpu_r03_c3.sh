#!/bin/bash
# r03 C3: range / point-polygon parity, the C3 line (the tree's library and explibs/ A/B),
# kernel stats, and the join tests + line (query row sort change)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py tests/test_gpu_callers.py \
  -m gpu -k "range or ppoly or join or q1 or mn_q1" -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/tests.log; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
P="python bench.py --workload ppoly --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $P > $O/ppoly.log 2>&1 && \
GF_LIB_PATH=explibs/lib_c3old.so timeout -k 10 200 $P --no-verify > $O/ppoly_old.log 2>&1 && \
timeout -k 10 200 $P --no-verify > $O/ppoly2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python -u bench.py --workload ppoly --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $O/prof.log 2>&1 && \
timeout -k 10 200 python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline > $O/join_u.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/jprof -o j --output-format csv -- python -u bench.py --workload join --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $O/jprof.log 2>&1
