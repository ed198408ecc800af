#!/bin/bash
# Host ASan + UBSan run of the product's host code on the GPU box (Makefile target asan-gpu, built
# on the CPU first: explibs/asan_gpu/).  The device code is the ordinary gfx950 code.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  tools/gpu_step.sh asan_driver 300 explibs/asan_gpu/asan_driver || exit 1
grep -q "asan_driver: ok" gpurun_out/asan_driver.log
