#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_geo 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_csv.py tests/test_gpu_geojson.py || exit 1
tools/gpu_step.sh b_geo 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --no-cpu-baseline || exit 1
tools/gpu_step.sh b_csv 300 python -u bench.py --workload csv --steps 20 --warmup 3 --no-cpu-baseline || exit 1
