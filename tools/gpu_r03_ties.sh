#!/bin/bash
# r03: tie-refined select + queued k > 512 tests, then the kNN / polygon kNN / range lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ties; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_knn_ties.py tests/test_gpu_polyknn.py tests/test_gpu_knn_large.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/knn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload polyknn --steps 30 --warmup 5 --cpu-seconds 5 > $O/polyknn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload range --points 1000000 --steps 192 --warmup 48 --no-cpu-baseline > $O/range1m.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload range --points 10000000 --steps 60 --warmup 12 --no-cpu-baseline > $O/range10m.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload ppoly --steps 30 --warmup 6 --no-cpu-baseline > $O/ppoly.log 2>&1 || exit 1
grep -h '^{' $O/*.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'], d['ms_per_step'], d['value'], d.get('verified_vs_oracle'), d.get('breakdown'))"
