# r03 join A/B on one box: the pre-rework library (explibs/lib_prejoin.so: task regions + packing)
# vs the chunked output at several chunk sizes; uniform C4, probe / bucket breakdown per line.
cd $GRAFT_REPO_ROOT
J="python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline --no-verify"
GF_LIB_PATH=explibs/lib_prejoin.so timeout -k 10 120 $J > gpurun_out/r03_ab_old.log 2>&1 && \
timeout -k 10 120 $J > gpurun_out/r03_ab_def.log 2>&1 && \
GF_JOIN_CHUNK=4096 timeout -k 10 120 $J > gpurun_out/r03_ab_c4k.log 2>&1 && \
GF_JOIN_CHUNK=65536 timeout -k 10 120 $J > gpurun_out/r03_ab_c64k.log 2>&1
