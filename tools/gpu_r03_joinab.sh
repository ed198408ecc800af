# r03 join A/B on one box, uniform C4 (probe / bucket breakdown per line):
#   old   explibs/lib_prejoin.so   r02's task regions + packing
#   wave  explibs/lib_blockchunks.so with GF_JOIN_WAVE_CHUNKS=1: one device atomic per wave chunk
#   blk   explibs/lib_blockchunks.so: a block's waves share its chunks
#   cur   the tree's library (block chunks + y-only histogram + step-end flushes), verified
#   cur64 the same with 64K-pair chunks
cd $GRAFT_REPO_ROOT
J="python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline"
GF_LIB_PATH=explibs/lib_prejoin.so timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_old.log 2>&1 && \
GF_LIB_PATH=explibs/lib_blockchunks.so GF_JOIN_WAVE_CHUNKS=1 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_wave.log 2>&1 && \
GF_LIB_PATH=explibs/lib_blockchunks.so timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_blk.log 2>&1 && \
timeout -k 10 180 $J > gpurun_out/r03_ab_cur.log 2>&1 && \
GF_JOIN_CHUNK=65536 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_cur64.log 2>&1
