#!/bin/bash
# round-5 polygon kNN refine experiments (DESIGN.md "Polygon-query kNN", r05 table: none kept).
# Runs the polygon kNN / tie GPU tests, then the bench line's kernel trace (launch interval:
# tools/trace_interval.py), then the line itself at depths 3 and 4, verified against the oracle.
# On the committed code it measures the baseline (separate refine launch, 30.1 us at depth 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_pk 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_polyknn.py tests/test_gpu_knn_ties.py || exit 1
grep -q " passed" gpurun_out/t_pk.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_pk.log || exit 1
$S pk_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pk_trace -o trace --output-format csv -- python -u bench.py --workload polyknn --steps 200 --warmup 10 --no-cpu-baseline --no-verify || exit 1
python tools/trace_interval.py gpurun_out/pk_trace/trace_kernel_trace.csv knn_poly_fused 10
for d in 3 4; do
  $S pk_d$d 300 python -u bench.py --workload polyknn --steps 200 --warmup 10 --pipeline $d --cpu-seconds 2 || exit 1
done
for f in gpurun_out/pk_d*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"), json.dumps(d.get("breakdown"))[:200])')"
done
