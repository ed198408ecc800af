#!/bin/bash
# round-5 GeoJSON byte-step unroll at 192-line blocks: 2 (the product) vs 1 / 4 (explibs/gu1, gu4:
# tools/build_exp.sh guN k_csv.hip "-DGF_GEO_UNROLL=N"), bench line A/B on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=gu5 bash tools/gpu_ab.sh "--workload geojson --steps 10 --warmup 2" gu1 gu4 || exit 1
