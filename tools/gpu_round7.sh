#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
tools/gpu_step.sh bench 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 3
tools/gpu_step.sh bench_t1 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-verify --timing-period 1
tools/gpu_step.sh bench_t1000 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-verify --timing-period 1000
tools/gpu_step.sh bench_s200 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-verify
tools/gpu_step.sh prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o fused --output-format csv -- python -u bench.py --steps 50 --warmup 10 --no-verify --no-cpu-baseline
tools/gpu_step.sh pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_fused -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python -u bench.py --steps 10 --warmup 4 --no-verify --no-cpu-baseline
tools/gpu_step.sh pmc_write 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn_fused -d gpurun_out/pmc_write -o write --output-format csv -- python -u bench.py --steps 10 --warmup 4 --no-verify --no-cpu-baseline
for f in bench bench_t1 bench_t1000 bench_s200; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['breakdown'])"; done
