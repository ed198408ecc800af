#!/bin/bash
# Run ONE GPU step under its own time limit; stop the whole call after a timeout, kill,
# abort or segfault (exit 124/137/134/139 or any signal), keep going after ordinary failures.
# usage: tools/gpu_step.sh NAME SECONDS cmd args...
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc in $(( $(date +%s) - start ))s"
tail -n 5 "gpurun_out/$name.log"
if [ $rc -ge 124 ]; then echo "[$name] fatal exit $rc: stopping this call"; exit $rc; fi
exit 0
