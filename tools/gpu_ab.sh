#!/bin/bash
# A/B on ONE box: the product library against experiment libraries (tools/build_exp.sh NAME SRC
# "-DDEFINES": explibs/NAME/libgeoflink_hip.so, selected with GF_LIB_PATH), the same bench command,
# arms interleaved twice.  PROF=1 adds a rocprofv3 --kernel-trace --stats run per arm (per-kernel
# times of phase-cost experiment builds: GF_BAND_EXP_*, GF_RANGE_EXP, GF_RADIX_EXP ...).
# usage: tools/gpu_ab.sh "bench.py args" [EXPLIB ...]        (round A/Bs of DESIGN.md §3 / §6)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
args=$1; shift
tag=${TAG:-ab}
for rep in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=explibs/$v/libgeoflink_hip.so
    GF_LIB_PATH=$lib $S ${tag}_${v}_$rep 400 python -u bench.py $args --no-cpu-baseline --no-verify || exit 1
    if [ "${PROF:-0}" = 1 ] && [ $rep = 1 ]; then
      GF_LIB_PATH=$lib $S ${tag}_p_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_p_$v -o stats \
        --output-format csv -- python -u bench.py $args --no-cpu-baseline --no-verify || exit 1
    fi
  done
done
for f in gpurun_out/${tag}_*_[12].log; do
  echo "$f $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], json.dumps(d.get("breakdown")))')"
done
