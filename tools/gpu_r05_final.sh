#!/bin/bash
# round-5 final evidence, part 1: host-ASan driver, PMC of the lines whose kernels changed late in
# the round (CSV, GeoJSON, C1 1M), the default bench line, the C2 launch trace and every workload
# line (tools/gpu_evidence.sh).  Part 2 is tools/gpu_suite.sh (smoke + the whole GPU suite).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_asan.sh || exit 1
ROUND=r05 bash tools/gpu_pmc_round.sh csv geojson range1m || exit 1
bash tools/gpu_evidence.sh
