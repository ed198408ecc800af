#!/bin/bash
# range (C3) kernel variants from _exp/ (GF_LIB_PATH): kernel stats each
export TMPDIR=/tmp
for v in "$@"; do
  GF_LIB_PATH=$PWD/_exp/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rexp_$v -o r --output-format csv -- python -u bench.py --workload ppoly --steps 10 --warmup 2 --no-verify --no-cpu-baseline --range-streams 1 > gpurun_out/rexp_$v.log 2>&1 || exit 1
  echo "$v done"
done
