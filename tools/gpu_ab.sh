#!/bin/bash
# The one A/B entry point: arms listed in a variants file, run on ONE box,
# interleaved REPS times (default 2), each arm's bench line collected into gpurun_out/<TAG>_ab.jsonl.
#
# usage: tools/gpu_ab.sh tools/ab/<name>.txt
# variants file, one arm per line ('#' comments), four '|'-separated fields:
#   NAME | ENV (K=V ..., or -) | LIB (explibs/<LIB>/libgeoflink_hip.so from tools/build_exp.sh, or -) | bench.py args
# options (environment):
#   REPS=n      interleaved repetitions (2)
#   PROF=1      one rocprofv3 --kernel-trace --stats run per arm (first repetition)
#   VERIFY=1    bench lines verified against the oracle (default --no-verify)
#   TESTS="..." pytest node ids run once per arm with an experiment library (GF_TEST_EXPERIMENT=1),
#               so an arm is parity-checked before it becomes the product
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=tools/gpu_step.sh
vfile=$1
[ -f "$vfile" ] || { echo "usage: $0 VARIANTS_FILE"; exit 2; }
tag=$(basename "$vfile" .txt)
reps=${REPS:-2}
q="--no-cpu-baseline"; [ "${VERIFY:-0}" = 1 ] || q="$q --no-verify"
mapfile -t arms < <(grep -v '^\s*#' "$vfile" | grep -v '^\s*$')
field() { echo "$1" | cut -d'|' -f"$2" | sed 's/^ *//; s/ *$//'; }
run_arm() {  # arm step-name kind(bench|prof|test)
  local a=$1 name=$2 kind=$3
  local envs lib args libpath=""
  envs=$(field "$a" 2); lib=$(field "$a" 3); args=$(field "$a" 4)
  [ "$envs" = "-" ] && envs=""
  [ "$lib" != "-" ] && libpath=explibs/$lib/libgeoflink_hip.so
  case $kind in
    bench) env $envs GF_LIB_PATH=$libpath $S "$name" 400 python -u bench.py $args $q ;;
    prof)  env $envs GF_LIB_PATH=$libpath $S "$name" 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o stats \
             --output-format csv -- python -u bench.py $args $q ;;
    test)  env $envs GF_LIB_PATH=$libpath GF_TEST_EXPERIMENT=1 $S "$name" 600 python -u -m pytest -x -q --timeout 200 \
             --timeout-method thread -p no:cacheprovider $TESTS ;;
  esac
}
if [ -n "$TESTS" ]; then
  for a in "${arms[@]}"; do
    [ "$(field "$a" 3)" = "-" ] && continue
    run_arm "$a" "${tag}_t_$(field "$a" 1)" test || exit 1
    grep -q " passed" "gpurun_out/${tag}_t_$(field "$a" 1).log" && ! grep -q "FAILED\|ERROR" "gpurun_out/${tag}_t_$(field "$a" 1).log" || exit 1
  done
fi
for rep in $(seq 1 "$reps"); do
  for a in "${arms[@]}"; do
    n=$(field "$a" 1)
    run_arm "$a" "${tag}_${n}_$rep" bench || exit 1
    if [ "${PROF:-0}" = 1 ] && [ "$rep" = 1 ]; then run_arm "$a" "${tag}_p_$n" prof || exit 1; fi
  done
done
out=gpurun_out/${tag}_ab.jsonl
: > "$out"
for a in "${arms[@]}"; do
  n=$(field "$a" 1)
  for rep in $(seq 1 "$reps"); do
    grep -h '^{' "gpurun_out/${tag}_${n}_$rep.log" | tail -1 | python -c '
import json, sys
d = json.loads(sys.stdin.read()); d["arm"] = sys.argv[1]; d["rep"] = int(sys.argv[2])
print(json.dumps(d))
print(sys.argv[1], sys.argv[2], d["ms_per_step"], json.dumps(d.get("breakdown"))[:160], file=sys.stderr)' "$n" "$rep" >> "$out"
  done
done
