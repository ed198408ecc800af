#!/bin/bash
# join variants (experiment libraries under _exp/, selected with GF_LIB_PATH): kernel stats each
export TMPDIR=/tmp
for v in "$@"; do
  GF_LIB_PATH=$PWD/_exp/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/jexp_$v -o j --output-format csv -- python -u bench.py --workload join --steps 5 --warmup 1 --no-verify --no-cpu-baseline > gpurun_out/jexp_$v.log 2>&1 || exit 1
  echo "$v done"
done
