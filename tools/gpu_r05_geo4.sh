#!/bin/bash
# round-5 GeoJSON experiment (not kept; the variant is not in the product): lanes taking the
# block's next line from an LDS queue when theirs ends (a build with that pass, run as "base"
# here) vs one line per lane (explibs/nobal, = the product): the ingest GPU tests, the bench line
# A/B on one box, kernel statistics.  Result: 3.08 vs 2.89 ms per 1M lines (GeoJSON).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_geo 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_csv.py tests/test_gpu_geojson.py tests/test_shim_native.py -k "csv or geojson or parse" || exit 1
grep -q " passed" gpurun_out/t_geo.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_geo.log || exit 1
TAG=gb bash tools/gpu_ab.sh "--workload geojson --steps 10 --warmup 2" nobal || exit 1
$S geo_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/geo_prof -o stats --output-format csv -- python -u bench.py --workload geojson --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
grep -h "csv_parse" gpurun_out/geo_prof/stats_kernel_stats.csv || true
