#!/bin/bash
# every SURVEY §8 configuration's single-GPU line (tools/bench_workloads.py) + kernel stats
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wl
mkdir -p $O
tools/gpu_step.sh wl_knn 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 5
tools/gpu_step.sh wl_range 300 python -u bench.py --workload range --steps 100 --warmup 10
tools/gpu_step.sh wl_ppoly 300 python -u bench.py --workload ppoly --steps 30 --warmup 5
tools/gpu_step.sh wl_join 300 python -u bench.py --workload join --steps 10 --warmup 2
tools/gpu_step.sh wl_sliding 400 python -u bench.py --workload sliding --steps 20 --warmup 4 --cpu-seconds 5
tools/gpu_step.sh wl_csv 300 python -u bench.py --workload csv --steps 20 --warmup 3 --cpu-seconds 5
tools/gpu_step.sh wl_polyknn 300 python -u bench.py --workload polyknn --steps 30 --warmup 5
tools/gpu_step.sh wl_pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3
tools/gpu_step.sh wl_geojson 300 python -u bench.py --workload geojson --steps 20 --warmup 3 --cpu-seconds 5
tools/gpu_step.sh wl_bucket 300 python -u bench.py --workload bucket --steps 20 --warmup 3
tools/gpu_step.sh wl_knn_cl 300 python -u bench.py --clustered --steps 20 --warmup 5 --cpu-seconds 5
tools/gpu_step.sh wl_join_cl 400 python -u bench.py --workload join --clustered --steps 5 --warmup 2
for w in range ppoly join csv polyknn pjoin geojson bucket; do
  tools/gpu_step.sh st_$w 300 rocprofv3 --kernel-trace --stats -d $O/$w -o $w --output-format csv -- python -u bench.py --workload $w --steps 5 --warmup 1 --no-verify --no-cpu-baseline
done
tools/gpu_step.sh st_knn 300 rocprofv3 --kernel-trace --stats -d $O/knn -o knn --output-format csv -- python -u bench.py --steps 200 --warmup 10 --no-verify --no-cpu-baseline
tools/gpu_step.sh st_sliding 300 rocprofv3 --kernel-trace --stats -d $O/sliding -o sliding --output-format csv -- python -u bench.py --workload sliding --steps 6 --warmup 2 --no-verify --no-cpu-baseline
python tools/trace_interval.py $O/knn/knn_kernel_trace.csv knn_fused 20 > $O/knn_interval.txt || true
grep -h '^{' gpurun_out/wl_*.log > $O/lines.jsonl || true
wc -l $O/lines.jsonl
