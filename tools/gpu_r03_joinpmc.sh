#!/bin/bash
# r03 join: parity of every join path, the uniform line, then rocprofv3 PMC passes over every
# join kernel (tools/gpu_pmc.sh: fetch / write / lds / occ / mem) summarised by tools/pmc_table.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/jp; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_clustered.py tests/test_gpu_sharding.py \
  -m gpu -k "join" -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/tests.log; tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline > $O/join_u.log 2>&1 || exit 1
PASSES="fetch write lds occ mem" tools/gpu_pmc.sh r03_join "join_|scan1" --workload join --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
python tools/pmc_table.py $O/join_pmc.json gpurun_out/pmc/r03_join --note "r03 join (band probe): bench.py --workload join --steps 5 --warmup 2"
