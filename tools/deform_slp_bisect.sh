#!/bin/bash
# Diagnostic builds of deform.o for the packed-fp32 co-residency fault: SLP
# vectorisation on (the build that failed), with the compiler's wait states padded (every instruction
# preceded by s_nop), or with every s_waitcnt forced to zero.  Usage (here, CPU): tools/deform_slp_bisect.sh
# Output: 4dlangsplat_amd/build/variants/liblsr_<name>.so; run tools/deform_race.py with LSR_LIBRARY=...
set -e
cd "$(dirname "$0")/../4dlangsplat_amd/csrc"
make -s -j8
OBJ=../build/obj; OUT=../build/variants; mkdir -p $OUT/obj
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics"
build() {   # name, extra flags...
    local name=$1; shift
    /opt/rocm/bin/hipcc $FLAGS "$@" -c -o $OUT/obj/deform_$name.o deform.hip 2>/dev/null
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liblsr_$name.so $(ls $OBJ/*.o | grep -v "/deform.o") $OUT/obj/deform_$name.o
    echo "built $OUT/liblsr_$name.so"
}
# results (round 5, tools/gpu.sh race): slp, slp_pad1 and slp_pad2 corrupt (pad: more rows);
# slp_wz faulted in the forward (illegal address) and is not built any more
[ -z "$ONLY" ] && build slp
[ "$ONLY" = slp ] && { build slp; exit 0; }
[ "$ONLY" = slp_bcast_asm ] && { build slp_bcast_asm -DLSR_FEAT_BCAST_ASM; exit 0; }
build slp_pad1 -Xarch_device -mllvm=-amdgpu-snop-padding=1
build slp_pad2 -Xarch_device -mllvm=-amdgpu-snop-padding=2
build slp_feat_scalar -DLSR_FEAT_SCALAR
# round 5, second level: which part of features_to_lds (bilinear weights, tap sums, plane product)
build slp_feat_w -DLSR_FEAT_SCALAR_W
build slp_feat_sum -DLSR_FEAT_SCALAR_SUM
build slp_feat_prod -DLSR_FEAT_SCALAR_PROD
# the weights as the SLP build's broadcast products, but never in place (inline asm, early clobber)
build slp_bcast_asm -DLSR_FEAT_BCAST_ASM
