#!/bin/bash
# round-5 final evidence, second pass (after the GeoJSON 192-line blocks and C3's two-lane drain):
# PMC + kernel statistics of the two changed lines, the default bench line, the C2 launch trace
# and every workload line (tools/gpu_evidence.sh).  The GPU suite follows in its own call
# (tools/gpu_suite.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=r05 bash tools/gpu_pmc_round.sh ppoly geojson || exit 1
bash tools/gpu_evidence.sh
