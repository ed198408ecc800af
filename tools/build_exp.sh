#!/bin/bash
# Experiment build of the product library with extra defines on ONE source file, linked with the
# regular objects of the others: explibs/<name>/libgeoflink_hip.so (select it with GF_LIB_PATH).
# Never the product: experiment defines break results on purpose (timing what a phase costs).
# The unit is compiled with -DGF_EXPERIMENT_BUILD, so gf_build_info() / gf_build_is_product()
# report it and the smoke / GPU suite refuse the library.
# usage: tools/build_exp.sh NAME SOURCE.hip "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; defs=$3
make -s build/obj/$(basename $src).o spatialflink_amd/libgeoflink_hip.so
mkdir -p explibs/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
  -Wno-unused-result -Wno-unused-value -DGF_EXPERIMENT_BUILD $defs -x hip -c spatialflink_amd/csrc/$src -o explibs/$name/$(basename $src).o
objs=$(ls build/obj/*.o | grep -v "/$(basename $src).o$")
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o explibs/$name/libgeoflink_hip.so $objs explibs/$name/$(basename $src).o
rm -f explibs/$name/*.o
echo "explibs/$name/libgeoflink_hip.so"
