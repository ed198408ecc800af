#!/bin/bash
# point-polygon join: parity tests, C3-shaped bench line + kernel stats; 2-rank gloo rehearsal of
# the N>1 range / ppoly / join / pjoin bench paths on one GPU (correctness of the plumbing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tools/gpu_step.sh gputests 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "join_ppoly" || exit 1
grep -q " passed" gpurun_out/gputests.log && ! grep -q "FAILED\|ERROR" gpurun_out/gputests.log || exit 1
tools/gpu_step.sh pjoin 300 python -u bench.py --workload pjoin --steps 20 --warmup 3 || exit 1
mkdir -p gpurun_out/pj
tools/gpu_step.sh st_pjoin 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pj -o pjoin --output-format csv -- python -u bench.py --workload pjoin --steps 10 --warmup 2 --no-verify || exit 1
for w in ppoly join pjoin range; do
  tools/gpu_step.sh mr_$w 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --workload $w --dist-backend gloo --points 2000000 --steps 5 --warmup 2 || exit 1
done
grep -h '^{' gpurun_out/pjoin.log gpurun_out/mr_*.log
