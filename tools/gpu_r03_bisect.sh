#!/bin/bash
# r03: which join commit broke test_join_clustered[500-0.004] / test_join_shards_with_query_halo:
# the failing tests against libraries built at earlier commits (explibs/, GF_LIB_PATH), then the
# uniform C4 join line at HEAD with its kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/bisect
T="tests/test_gpu_clustered.py tests/test_gpu_sharding.py -m gpu -k join -q --timeout 200 --timeout-method thread -x"
for c in 6b29cde 54dad06 837e03d; do
  GF_LIB_PATH=explibs/lib_$c.so timeout -k 10 400 python -u -m pytest $T > gpurun_out/bisect/$c.log 2>&1; rc=$?
  echo "$c rc=$rc" | tee -a gpurun_out/bisect/summary.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 200 python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bisect/join_u.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bisect/prof -o join --output-format csv -- python -u bench.py --workload join --steps 10 --warmup 3 --no-cpu-baseline --no-verify > gpurun_out/bisect/join_prof.log 2>&1
