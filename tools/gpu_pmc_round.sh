#!/bin/bash
# Per-round PMC + kernel-stats campaign over the final kernels of every workload line (VERDICT r02
# item 2).  Per workload: one `rocprofv3 --kernel-trace --stats` run, then one --pmc run per
# counter group (tools/gpu_pmc.sh: FETCH_SIZE and WRITE_SIZE never share a pass), summarised by
# tools/pmc_table.py into gpurun_out/pmc_${ROUND}/<tag>.json -> copied to profiles/${ROUND}_<tag>_pmc.json.
# usage: ROUND=r04 tools/gpu_pmc_round.sh TAG... (default: all)   tags: knn range1m range10m ppoly join
#        joinc pjoin sliding bucket csv geojson polyknn
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
COMMON="--steps 5 --warmup 2 --no-cpu-baseline --no-verify"
OUT=gpurun_out/pmc_${ROUND}
mkdir -p $OUT
one() {  # tag kernel-regex passes bench-args...
  local tag=$1 re=$2 passes=$3; shift 3
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/$tag/stats -o stats --output-format csv \
    -- python -u bench.py "$@" $COMMON > $OUT/$tag.stats.log 2>&1 || { echo "[stats $tag] failed"; tail -5 $OUT/$tag.stats.log; exit 1; }
  PASSES="$passes" tools/gpu_pmc.sh "${ROUND}_$tag" "$re" "$@" $COMMON
  python tools/pmc_table.py $OUT/$tag.json gpurun_out/pmc/${ROUND}_$tag --note "${ROUND} $tag: $* $COMMON"
  cp $OUT/$tag/stats/*kernel_stats.csv $OUT/${tag}_kernel_stats.csv 2>/dev/null || true
  echo "[campaign $tag] ok"
}
TAGS=${*:-knn range1m range10m ppoly join joinc pjoin sliding bucket csv geojson polyknn}
for t in $TAGS; do
  case $t in
    knn)      one knn "knn_fused|knn_sample" "fetch write occ" ;;
    range1m)  one range1m "range_batch|range_kernel|expand" "fetch write occ" --workload range --points 1000000 ;;
    range10m) one range10m "range_kernel|expand" "fetch write occ" --workload range --points 10000000 ;;
    ppoly)    one ppoly "range_kernel|range_test|expand" "fetch write lds occ" --workload ppoly ;;
    join)     one join "join_|scan1" "fetch write lds occ mem" --workload join ;;
    joinc)    one joinc "join_band" "write lds occ mem" --workload join --clustered ;;
    pjoin)    one pjoin "range_kernel|join_ppoly" "fetch write occ" --workload pjoin ;;
    sliding)  one sliding "knn_fused|knn_merge|pane_bounds" "fetch write occ" --workload sliding ;;
    bucket)   one bucket "radix|scan1|assign" "fetch write lds occ" --workload bucket ;;
    csv)      one csv "csv_" "fetch write occ" --workload csv ;;
    geojson)  one geojson "csv_|geo" "fetch write lds occ" --workload geojson ;;
    polyknn)  one polyknn "knn_poly|knn_select" "fetch write occ" --workload polyknn ;;
  esac
done
