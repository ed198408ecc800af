#!/bin/bash
# r03: broadcast-rank select -- kNN parity tests, select phase trace (point and polygon), lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sel; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_knn_ties.py tests/test_gpu_polyknn.py tests/test_gpu_knn_large.py tests/test_gpu_sliding.py tests/test_gpu_parity.py -k "knn or sliding or merge or ties or poly" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GF_LIB_PATH=$PWD/explibs/trace.so timeout -k 10 200 python -u tools/trace_select.py > $O/trace_point.log 2>&1 || exit 1
GF_LIB_PATH=$PWD/explibs/trace.so POLY=1 timeout -k 10 200 python -u tools/trace_select.py > $O/trace_poly.log 2>&1 || exit 1
cat $O/trace_point.log $O/trace_poly.log | grep -v amdgpu.ids
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/knn_$rep.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --workload polyknn --steps 30 --warmup 5 --no-cpu-baseline > $O/polyknn.log 2>&1 || exit 1
grep -h '^{' $O/knn_*.log $O/polyknn.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'], d['ms_per_step'], d['value'], d.get('verified_vs_oracle'), d.get('breakdown'))"
