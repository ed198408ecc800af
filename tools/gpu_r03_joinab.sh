# r03 join A/B on one box, uniform C4 (probe / bucket breakdown per line): the pre-rework library
# (explibs/lib_prejoin.so: task regions + packing), wave chunks (GF_JOIN_WAVE_CHUNKS=1) at two
# chunk sizes, and block chunks (the default, verified against the oracle) at three.
cd $GRAFT_REPO_ROOT
J="python bench.py --workload join --steps 20 --warmup 5 --no-cpu-baseline"
GF_LIB_PATH=explibs/lib_prejoin.so timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_old.log 2>&1 && \
GF_JOIN_WAVE_CHUNKS=1 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_wave.log 2>&1 && \
GF_JOIN_WAVE_CHUNKS=1 GF_JOIN_CHUNK=8192 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_wave8k.log 2>&1 && \
timeout -k 10 180 $J > gpurun_out/r03_ab_block.log 2>&1 && \
GF_JOIN_CHUNK=4096 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_block4k.log 2>&1 && \
GF_JOIN_CHUNK=65536 timeout -k 10 120 $J --no-verify > gpurun_out/r03_ab_block64k.log 2>&1
