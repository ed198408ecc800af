#!/bin/bash
# r03 A/B: C3 / C1 span-prefilter scan with the 192-entry wave queue (explibs/head.so) and the
# 128-entry queue with split tile pushes (in-tree); range parity tests on the in-tree library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/abc3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "range or ppoly" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in head new; do
    if [ $v = new ]; then unset GF_LIB_PATH; else export GF_LIB_PATH=$PWD/explibs/$v.so; fi
    timeout -k 10 120 python -u bench.py --workload ppoly --steps 60 --warmup 9 --no-cpu-baseline --no-verify > $O/c3_${v}_$rep.log 2>&1 || exit 1
    timeout -k 10 120 python -u bench.py --workload ppoly --steps 60 --warmup 9 --no-cpu-baseline --no-verify --range-streams 1 > $O/c3s1_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -h '^{' $O/c3_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['scan_us'])") single-stream $(grep -h '^{' $O/c3s1_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['scan_us'])")"
  done
done
