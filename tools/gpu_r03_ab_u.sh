#!/bin/bash
# r03 A/B: range scan tiles per wave iteration U = 2 (in-tree) / 3 / 4 (explibs/u3.so, u4.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/abu; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-verify"
for rep in 1 2; do
  for v in u2 u3 u4; do
    if [ $v = u2 ]; then unset GF_LIB_PATH; else export GF_LIB_PATH=$PWD/explibs/$v.so; fi
    timeout -k 10 120 $B --workload range --points 10000000 --steps 300 --warmup 30 > $O/r10_${v}_$rep.log 2>&1 || exit 1
    timeout -k 10 120 $B --workload range --points 1000000 --steps 800 --warmup 48 > $O/r1_${v}_$rep.log 2>&1 || exit 1
    if [ $v != u4 ]; then timeout -k 10 120 $B --workload ppoly --steps 300 --warmup 30 > $O/c3_${v}_$rep.log 2>&1 || exit 1; fi
    echo "$v $rep r10 $(grep -h '^{' $O/r10_${v}_$rep.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") r1 $(grep -h '^{' $O/r1_${v}_$rep.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") c3 $(grep -h '^{' $O/c3_${v}_$rep.log 2>/dev/null | python -c "import json,sys; t=sys.stdin.read(); print(json.loads(t)['ms_per_step'] if t.strip() else '-')")"
  done
done
