#!/bin/bash
# libocf variant with ocf_tiles.hip compiled under extra -D switches (timing probes): the other objects are the
# normal build's.   bash tools/build_variant.sh NAME "-DOCF_ET_NOMFMA ..."  ->  .../libocf_NAME.so
set -e
C=$(dirname "$0")/../omnidirectional_collaborative_filtering_amd/csrc
cd "$C"
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
  -munsafe-fp-atomics $2 -c ocf_tiles.hip -o build_var/ocf_tiles_$1.o
objs=$(ls build/*.o | grep -v ocf_tiles.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build_var/ocf_tiles_$1.o -o ../libocf_$1.so
