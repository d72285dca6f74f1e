// lsr_mfma.h -- matrix-core helpers of the compositor backward (render_bwd_wave.hip).
//
// v_mfma_f32_16x16x32_bf16 lane maps (checked bit-exactly by tests/kernels/t_mfma16.hip):
//   A (16 x 32): lane l holds A[l & 15][8 (l >> 4) + j], j = 0..7
//   B (32 x 16): lane l holds B[8 (l >> 4) + j][l & 15]
//   D (16 x 16): lane l, register i holds D[4 (l >> 4) + i][l & 15]
// fp32 accuracy from bf16 inputs: x = hi + lo with hi = bf16(x), lo = bf16(x - hi); a product
// a*b is taken as ah*bh + ah*bl + al*bh (three MFMAs, ~2^-17 relative, fp32 accumulation).
#pragma once
#include <hip/hip_runtime.h>

namespace lsr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LSR_MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}

// ds_read_b64_tr_b16: each 16-lane group reads a 4-row x 16-column block of 16-bit values; lane i
// of the group supplies the address of row (i >> 2), columns 4 (i & 3) .. +3 and receives column
// i of the block (its 4 rows).
__device__ __forceinline__ bf16x4 ds_read_tr16(const __bf16* p) {
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4*>(reinterpret_cast<size_t>(p)));
    return __builtin_bit_cast(bf16x4, v);
}

// 4 x 4 transpose across the four 16-lane groups: on entry lane group g holds x[p] (p = 0..3);
// on exit lane group g holds, in x[p], what group p held in x[g] (same lane within the group).
// Two permlane32 swaps then two permlane16 swaps.
__device__ __forceinline__ void transpose_lane_groups(float (&x)[4]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[p]), __float_as_uint(x[p + 2]), false, false);
        x[p] = __uint_as_float(r[0]);
        x[p + 2] = __uint_as_float(r[1]);
    }
#pragma unroll
    for (int p = 0; p < 4; p += 2) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[p]), __float_as_uint(x[p + 1]), false, false);
        x[p] = __uint_as_float(r[0]);
        x[p + 1] = __uint_as_float(r[1]);
    }
}

}  // namespace lsr
