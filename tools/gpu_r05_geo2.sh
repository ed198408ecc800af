#!/bin/bash
# round-5 GeoJSON parse occupancy / wave balance, as run (the product then had 256-line blocks and
# the length-order sort, GF_GEO_SORT=1, since removed): vs index order (explibs/nosort), 192 /
# 128-line blocks (explibs/g192, g128, g192ns = 192 without the sort).  tools/build_exp.sh NAME
# k_csv.hip "-DGF_GEO_LINES=N".  Result: 192 lines without the sort is the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_geo 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_csv.py tests/test_gpu_geojson.py tests/test_shim_native.py -k "csv or geojson or parse" || exit 1
grep -q " passed" gpurun_out/t_geo.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_geo.log || exit 1
$S geo_b1 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --no-cpu-baseline || exit 1
TAG=gs bash tools/gpu_ab.sh "--workload geojson --steps 10 --warmup 2" nosort g192 g128 g192ns || exit 1
$S geo_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/geo_prof -o stats --output-format csv -- python -u bench.py --workload geojson --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
grep -h "csv_parse" gpurun_out/geo_prof/stats_kernel_stats.csv || true
for f in gpurun_out/geo_b1.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"), json.dumps(d.get("breakdown"))[:200])')"
done
