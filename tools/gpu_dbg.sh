#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u tools/dbg_sliding.py > gpurun_out/dbg.log 2>&1; echo rc=$?
tail -60 gpurun_out/dbg.log
