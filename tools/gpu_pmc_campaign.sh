#!/bin/bash
# North-star PMC campaign (r02): FETCH/WRITE, LDS + VALU, occupancy/waits for the dominant
# kernel of each headline workload, one rocprofv3 pass per counter group (tools/gpu_pmc.sh),
# then tools/pmc_table.py summaries into profiles/r02_<tag>_pmc.json.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
COMMON="--steps 5 --warmup 2 --no-cpu-baseline --no-verify"
tools/gpu_pmc.sh knn   "knn_fused"                              $COMMON
tools/gpu_pmc.sh range "range_kernel|range_test|range_finalize" --workload range --points 10000000 $COMMON
tools/gpu_pmc.sh ppoly "range_kernel|range_test"                --workload ppoly $COMMON
tools/gpu_pmc.sh polyknn "knn_poly"                             --workload polyknn $COMMON
