#!/bin/bash
# round-5 join occupancy experiment: two band-probe blocks per CU.
#   base      the product (one 160 KB, 1024-thread block per CU: 4 waves / SIMD, 128 VGPRs)
#   base2     the product with two blocks per CU in the grid (GF_JOIN_BAND_PER_CU=2: two rounds)
#   jocc2     explibs/jocc (tools/build_exp.sh jocc k_join.hip "-DGF_BAND_LDS_KB=80
#             -DGF_BAND_MINBLK=2 -DGF_BAND_BUF=320"): 80 KB blocks, launch bounds for 8 waves / SIMD
#             (64 VGPRs), two per CU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --no-verify --workload join"
for rep in 1 2; do
  $S jo_base_$rep 300 $B --steps 20 --warmup 4 || exit 1
  GF_JOIN_BAND_PER_CU=2 $S jo_base2_$rep 300 $B --steps 20 --warmup 4 || exit 1
  GF_LIB_PATH=explibs/jocc/libgeoflink_hip.so GF_JOIN_BAND_PER_CU=2 $S jo_jocc2_$rep 300 $B --steps 20 --warmup 4 || exit 1
done
$S joc_base 300 $B --clustered --steps 4 --warmup 2 || exit 1
GF_LIB_PATH=explibs/jocc/libgeoflink_hip.so GF_JOIN_BAND_PER_CU=2 $S joc_jocc2 300 $B --clustered --steps 4 --warmup 2 || exit 1
GF_LIB_PATH=explibs/jocc/libgeoflink_hip.so GF_JOIN_BAND_PER_CU=2 $S jo_p_jocc2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jo_p_jocc2 -o stats --output-format csv -- $B --steps 20 --warmup 4 --join-streams 1 || exit 1
$S jo_p_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jo_p_base -o stats --output-format csv -- $B --steps 20 --warmup 4 --join-streams 1 || exit 1
for f in gpurun_out/jo_*_[12].log gpurun_out/joc_*.log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], json.dumps(d.get("breakdown")))')"
done
