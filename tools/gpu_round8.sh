#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log
tools/gpu_step.sh bench2_gloo 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --points 2000000
tools/gpu_step.sh bench2_gloo_p1 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --points 2000000 --pipeline 1 --exchange-batch 3
tools/gpu_step.sh tune 300 python -u tools/tune_fused.py
grep '^{' gpurun_out/bench2_gloo.log gpurun_out/bench2_gloo_p1.log
cat gpurun_out/tune.log
