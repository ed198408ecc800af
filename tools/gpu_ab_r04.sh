#!/bin/bash
# Round-4 A/B comparisons behind DESIGN.md's r04 notes, in one GPU call.  Experiment libraries
# first, on the CPU (tools/build_exp.sh; never the product -- their defines break results on
# purpose or select the older variant):
#   tools/build_exp.sh jp0 k_join.hip  "-DGF_BAND_PAIR=0"   # join probe: one point per walk
#   tools/build_exp.sh re1 k_range.hip "-DGF_RANGE_EXP=1"   # C3 without the classification rounds
#   tools/build_exp.sh rx5 k_points.hip "-DGF_RADIX_EXP=5"  # K2 pass-0 histogram without key stores
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
Q="--no-cpu-baseline --no-verify"
$S ab_k2_row 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
GF_K2_LSD=1 $S ab_k2_lsd 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
GF_RADIX_NT=1024 $S ab_k2_nt1024 200 python -u bench.py --workload bucket --steps 20 --warmup 3 || exit 1
$S ab_knn_d3 300 python -u bench.py --pipeline 3 --steps 30 --warmup 8 $Q || exit 1
$S ab_knn_d4 300 python -u bench.py --pipeline 4 --steps 30 --warmup 8 $Q || exit 1
$S ab_polyknn_d3 300 python -u bench.py --workload polyknn --pipeline 3 --steps 40 --warmup 8 $Q || exit 1
$S ab_polyknn_d4 300 python -u bench.py --workload polyknn --pipeline 4 --steps 40 --warmup 8 $Q || exit 1
$S ab_join_s1 300 python -u bench.py --workload join --join-streams 1 --steps 20 --warmup 3 $Q || exit 1
$S ab_join_s2 300 python -u bench.py --workload join --join-streams 2 --steps 20 --warmup 3 $Q || exit 1
$S ab_c3_blocks 300 python -u bench.py --workload ppoly --range-blocks 256,512,768,1024 --steps 300 --warmup 30 $Q || exit 1
for v in jp0 re1 rx5; do
  [ -f explibs/$v/libgeoflink_hip.so ] || continue
  case $v in jp0) w="--workload join --steps 20 --warmup 3";; re1) w="--workload ppoly --steps 100 --warmup 10";;
             rx5) w="--workload bucket --steps 20 --warmup 3";; esac
  GF_LIB_PATH=explibs/$v/libgeoflink_hip.so $S ab_exp_$v 300 python -u bench.py $w $Q || exit 1
done
