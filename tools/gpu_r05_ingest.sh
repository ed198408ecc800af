#!/bin/bash
# round-5 checks of the one-sync ingest (the line count read on the device) and the batched range
# grid: the ingest / range-batch GPU tests, then the CSV, GeoJSON and C1 1M bench lines verified
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_ingest 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_csv.py tests/test_gpu_geojson.py tests/test_shim_native.py "tests/test_gpu_parity.py" -k "csv or geojson or parse or batch or range" || exit 1
grep -q " passed" gpurun_out/t_ingest.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_ingest.log || exit 1
$S in_csv 300 python -u bench.py --workload csv --steps 20 --warmup 3 --cpu-seconds 2 || exit 1
$S in_geojson 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --no-cpu-baseline || exit 1
$S in_c1 300 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --cpu-seconds 2 || exit 1
$S in_csv_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/in_csv_prof -o stats --output-format csv -- python -u bench.py --workload csv --steps 20 --warmup 3 --no-cpu-baseline --no-verify || exit 1
for f in gpurun_out/in_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"), json.dumps(d.get("breakdown"))[:200])')"
done
