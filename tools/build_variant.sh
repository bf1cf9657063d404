#!/bin/bash
# libocf variant with one translation unit compiled under extra -D switches (timing probes / A/B): the other
# objects are the normal build's.   bash tools/build_variant.sh NAME SOURCE.hip "-DOCF_... ..."
#   -> omnidirectional_collaborative_filtering_amd/libocf_NAME.so
set -e
C=$(dirname "$0")/../omnidirectional_collaborative_filtering_amd/csrc
cd "$C"
mkdir -p build_var
src=${2%.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
  -munsafe-fp-atomics $3 -c $src.hip -o build_var/${src}_$1.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build_var/${src}_$1.o -o ../libocf_$1.so
