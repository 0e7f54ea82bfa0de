#!/bin/bash
# Device assembly of the library's HIP sources, comments and debug lines stripped, for an
# instruction-for-instruction comparison of two trees (e.g. before / after removing a build
# switch whose default is kept):
#   scripts/isa/dump_isa.sh OUTDIR [extra hipcc flags]   ->  OUTDIR/<file>.s
#   diff -r OUTDIR_before OUTDIR_after
set -e
out=$1; shift
mkdir -p "$out"
cd "$(dirname "$0")/../../my-nope-nerf_amd"
for f in csrc/*.hip; do
    b=$(basename "$f")
    extra=""
    case "$b" in gemm_x6.hip|wgrad.hip) extra="-fno-slp-vectorize" ;; esac
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $extra "$@" \
        --cuda-device-only -S "$f" -o - 2>/dev/null |
        grep -v -E '^\s*(;|\.loc|\.file|\.Ltmp|\.Ldebug|\.section\s+\.debug|\.ident|\.amdhsa_|\.p2align)' |
        sed -e 's/\s*;.*$//' > "$out/$b.s" &
done
wait
echo "assembly in $out"
