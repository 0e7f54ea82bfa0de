#!/bin/bash
# A diagnostic variant of the library with one source file rebuilt with extra defines, linked
# with the tree's other objects (my-nope-nerf_amd/build):
#   scripts/isa/variant_file.sh NAME FILE.hip -DFOO=1 ...  -> my-nope-nerf_amd/lib/ab/NAME.so
# (not committed; lib_ab.py / NERF_HIP_LIB take it)
set -e
cd "$(dirname "$0")/../../my-nope-nerf_amd"
name=$1; file=$2; shift 2
mkdir -p build_ab/$name lib/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c csrc/$file -o build_ab/$name/$file.o
objs=$(ls build/*.o | grep -v "/$file.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/ab/$name.so $objs build_ab/$name/$file.o
echo "built lib/ab/$name.so"
