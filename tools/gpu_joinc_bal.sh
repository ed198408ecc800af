cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for v in bal32 base; do
lib=""; [ -f explibs/$v/libgeoflink_hip.so ] && lib=explibs/$v/libgeoflink_hip.so
GF_LIB_PATH=$lib tools/gpu_step.sh bjc_$v 300 python -u bench.py --workload join --clustered --steps 5 --warmup 2 --no-cpu-baseline --no-verify || exit 1
done
