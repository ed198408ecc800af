#!/bin/bash
# round-5 join A/B: the product (flat run-select chain) against explibs/jnest (nested ?: select)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF=1 TAG=ju bash tools/gpu_ab.sh "--workload join --steps 20 --warmup 4" jnest && TAG=jc bash tools/gpu_ab.sh "--workload join --clustered --steps 4 --warmup 2" jnest
