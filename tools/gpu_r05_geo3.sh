#!/bin/bash
# round-5 GeoJSON 192-line blocks (the product default): the ingest GPU tests and the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_geo 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_csv.py tests/test_gpu_geojson.py tests/test_shim_native.py -k "csv or geojson or parse" || exit 1
grep -q " passed" gpurun_out/t_geo.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_geo.log || exit 1
for r in 1 2; do
  $S geo_b$r 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --no-cpu-baseline || exit 1
done
for f in gpurun_out/geo_b*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"), json.dumps(d.get("breakdown"))[:200])')"
done
