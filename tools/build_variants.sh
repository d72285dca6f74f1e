#!/bin/bash
# Ablation builds of liblsr.so for profiling experiments: each variant recompiles one source
# with extra -D flags and links it with the regular objects.  Usage:
#   tools/build_variants.sh name:source.hip:-DFLAG[,-DFLAG2] ...
# Output: 4dlangsplat_amd/build/variants/liblsr_<name>.so (select with LSR_LIBRARY=...).
set -e
cd "$(dirname "$0")/../4dlangsplat_amd/csrc"
make -s -j8
OBJ=../build/obj; OUT=../build/variants; mkdir -p $OUT/obj
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics"
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; defs=${rest#*:}; defs=${defs//,/ }
    base=${src%.hip}
    [ "$base" = preprocess ] && defs="$defs -fno-slp-vectorize"   # as in the Makefile
    [ "$base" = train ] && defs="$defs -fno-slp-vectorize"
    [ "$base" = deform ] && defs="$defs -fno-slp-vectorize"
    /opt/rocm/bin/hipcc $FLAGS $defs -c -o $OUT/obj/${base}_$name.o $src
    objs=$(ls $OBJ/*.o | grep -v "/$base.o")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liblsr_$name.so $objs $OUT/obj/${base}_$name.o
    echo "built $OUT/liblsr_$name.so"
done
