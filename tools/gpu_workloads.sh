#!/bin/bash
# every SURVEY §8 configuration's single-GPU line (bench.py / tools/bench_workloads.py), each
# verified against the oracle (or the whole-window evaluation), with its CPU baselines; the
# lines are collected into gpurun_out/wl/lines.jsonl (-> profiles/rNN_workloads.jsonl).  Kernel
# statistics and PMC of the same commands: tools/gpu_pmc_round.sh.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wl
mkdir -p $O
S=tools/gpu_step.sh
$S wl_knn 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 5
$S wl_range1m 300 python -u bench.py --workload range --points 1000000 --steps 800 --warmup 48 --cpu-seconds 5
$S wl_range10m 300 python -u bench.py --workload range --points 10000000 --steps 300 --warmup 30 --cpu-seconds 5
$S wl_ppoly 300 python -u bench.py --workload ppoly --steps 300 --warmup 30 --cpu-seconds 5
$S wl_join 300 python -u bench.py --workload join --steps 20 --warmup 5 --cpu-seconds 5
$S wl_sliding 400 python -u bench.py --workload sliding --steps 20 --warmup 4 --cpu-seconds 5
$S wl_csv 300 python -u bench.py --workload csv --steps 20 --warmup 3 --cpu-seconds 5
$S wl_polyknn 300 python -u bench.py --workload polyknn --steps 200 --warmup 10 --cpu-seconds 5
$S wl_pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 --cpu-seconds 5
$S wl_geojson 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --cpu-seconds 5
$S wl_bucket 300 python -u bench.py --workload bucket --steps 20 --warmup 3
$S wl_knn_cl 300 python -u bench.py --clustered --steps 20 --warmup 5 --cpu-seconds 5
$S wl_join_cl 400 python -u bench.py --workload join --clustered --steps 5 --warmup 2 --no-cpu-baseline
grep -h '^{' gpurun_out/wl_*.log > $O/lines.jsonl || true
wc -l $O/lines.jsonl
