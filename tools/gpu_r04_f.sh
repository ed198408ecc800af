#!/bin/bash
# r04: K2 scatter with the next tile loaded after placement; pass-0 histogram experiments; join
# probe walking a lane's two points as one sequence (vs explibs/jp0: one point at a time)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh t_f1 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_knn_large.py tests/test_gpu_sharding.py tests/test_gpu_join_density.py tests/test_gpu_clustered.py -k "bucket or knn_large or shard or join" || exit 1
tools/gpu_step.sh b_bucket 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh p_bucket 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bucket -o stats --output-format csv -- python -u bench.py --workload bucket --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh b_join 400 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline || exit 1
GF_LIB_PATH=explibs/jp0/libgeoflink_hip.so tools/gpu_step.sh b_join_jp0 400 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline --no-verify || exit 1
tools/gpu_step.sh p_join 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_join -o stats --output-format csv -- python -u bench.py --workload join --join-streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
for v in rx4 rx5; do
  GF_LIB_PATH=explibs/$v/libgeoflink_hip.so tools/gpu_step.sh px_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/px_$v -o stats --output-format csv -- python -u bench.py --workload bucket --steps 10 --warmup 2 --no-cpu-baseline --no-verify || exit 1
done
