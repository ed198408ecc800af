#!/bin/bash
# r03: polygon kNN windows in flight (--poly-streams 1 / 2 / 3), verified, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ps; mkdir -p $O
for rep in 1 2; do
  for s in 1 2 3; do
    timeout -k 10 150 python -u bench.py --workload polyknn --steps 200 --warmup 10 --no-cpu-baseline --poly-streams $s > $O/s${s}_$rep.log 2>&1 || { tail -20 $O/s${s}_$rep.log; exit 1; }
    echo "$s $rep $(grep -h '^{' $O/s${s}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['verified_vs_oracle'], d['fallback_windows'], d['breakdown'])")"
  done
done
