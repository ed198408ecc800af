#!/bin/bash
# round 5: join parity (density, clustered, parity -k join) then the uniform + clustered C4 lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_join 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_join_density.py tests/test_gpu_clustered.py tests/test_gpu_parity.py -k "join" || exit 1
grep -q " passed" gpurun_out/t_join.log && ! grep -q "FAILED\|ERROR" gpurun_out/t_join.log || exit 1
$S b_join 300 python -u bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline ${JOINARGS} || exit 1
$S b_join_cl 400 python -u bench.py --workload join --clustered --steps 5 --warmup 2 --no-cpu-baseline ${JOINARGS}
