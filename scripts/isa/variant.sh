#!/bin/bash
# A diagnostic variant of the library: chain.hip rebuilt with extra defines, linked with the
# tree's other objects (my-nope-nerf_amd/build): scripts/isa/variant.sh NAME -DFOO=1 ...
# -> my-nope-nerf_amd/lib/ab/NAME.so (not committed; lib_ab.py / NERF_HIP_LIB take it)
set -e
cd "$(dirname "$0")/../../my-nope-nerf_amd"
name=$1; shift
mkdir -p build_ab/$name lib/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c csrc/chain.hip -o build_ab/$name/chain.hip.o
objs=$(ls build/*.o | grep -v chain.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/ab/$name.so $objs build_ab/$name/chain.hip.o
echo "built lib/ab/$name.so"
