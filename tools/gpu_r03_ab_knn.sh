#!/bin/bash
# r03 A/B: headline kNN with the previous select (explibs/head.so), the tie-refined select
# (in-tree), and tie refinement only in the standalone select (explibs/nolite.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
  for v in head new nolite; do
    if [ $v = new ]; then unset GF_LIB_PATH; else export GF_LIB_PATH=$PWD/explibs/$v.so; fi
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-verify > $O/knn_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -h '^{' $O/knn_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown']['window_us'], d['breakdown']['select_us'], d['breakdown']['scan_us'])")"
  done
done
