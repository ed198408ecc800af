#!/bin/bash
# r03 A/B: K2 bucketing with 9-bit digits (2 passes at 500^2, in-tree) vs 6-bit (3 passes, explibs/b6.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/abb; mkdir -p $O
for rep in 1 2; do
  for v in b9 b6; do
    if [ $v = b9 ]; then unset GF_LIB_PATH; else export GF_LIB_PATH=$PWD/explibs/$v.so; fi
    timeout -k 10 150 python -u bench.py --workload bucket --steps 50 --warmup 5 > $O/${v}_$rep.log 2>&1 || exit 1
    timeout -k 10 150 python -u bench.py --workload bucket --steps 50 --warmup 5 --grid 1000 > $O/${v}_g1000_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep -h '^{' $O/${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['verified_vs_oracle'] if 'verified_vs_oracle' in d else d.get('verified'), d['breakdown']['kernel_us_per_window'])") g1000 $(grep -h '^{' $O/${v}_g1000_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('verified_vs_oracle', d.get('verified')))")"
  done
done
