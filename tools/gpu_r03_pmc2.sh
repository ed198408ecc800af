#!/bin/bash
# r03: PMC campaign part 2 (sliding, K2, CSV, GeoJSON, polygon kNN), then the query row sort's
# kernel stats with an experiment build that skips its sorted-copy stores (explibs/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_pmc_r03.sh sliding bucket csv geojson polyknn || exit 1
if [ -f explibs/lib_sortnostore.so ]; then
  GF_LIB_PATH=explibs/lib_sortnostore.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sortexp -o s --output-format csv \
    -- python -u bench.py --workload join --steps 10 --warmup 3 --no-cpu-baseline --no-verify > gpurun_out/sortexp.log 2>&1 || exit 1
fi
