cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tools/gpu_step.sh t_new 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_a_gpu_multirank.py tests/test_gpu_comm.py tests/test_shim_native.py tests/test_gpu_knn_ties.py || exit 1
tools/gpu_step.sh b_knn 200 python -u bench.py --steps 20 --warmup 5
