#!/bin/bash
# The product library of an earlier git revision, for A/B timing against the working tree on ONE
# box (tools/gpu_ab.sh: an arm whose LIB is NAME): explibs/NAME/libgeoflink_hip.so.
# usage: tools/build_rev.sh REV NAME          (e.g. tools/build_rev.sh HEAD~1 prev)
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
[ -n "$rev" ] && [ -n "$name" ] || { echo "usage: $0 REV NAME"; exit 2; }
tmp=$(mktemp -d /tmp/gfrev.XXXXXX)
git archive "$rev" spatialflink_amd/csrc include Makefile | tar -x -C "$tmp"
make -s -C "$tmp" -j8 spatialflink_amd/libgeoflink_hip.so OBJDIR=build/obj
mkdir -p explibs/$name
cp "$tmp/spatialflink_amd/libgeoflink_hip.so" explibs/$name/libgeoflink_hip.so
rm -rf "$tmp"
echo "explibs/$name/libgeoflink_hip.so ($(git rev-parse --short "$rev"))"
