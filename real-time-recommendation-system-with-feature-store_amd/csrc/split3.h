// fp32 products on the bf16 MFMA: the three-piece split shared by the tower
// kernels (mlp.hip) and the fp32 loss kernels (loss.hip); DESIGN.md §5 note i,
// bounds pinned on the host by tests/test_split3_cpu.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rt {
namespace fsplit {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// x = hi + mid + lo with each piece the RNE bf16 of what the previous pieces
// left (every residual is exact in fp32), |x - hi - mid - lo| <= 2^-24 |x|.
// A product x·y is taken as the 6 piece products of order <= 2^-16 (hi·hi,
// hi·mid, mid·hi, mid·mid, hi·lo, lo·hi); the 3 dropped ones are below
// 2^-23 |x·y|, and each piece product is exact in the MFMA's fp32 sum. So a
// 32x32x16 bf16 MFMA sextet does the work of 8 fp32 32x32x2 MFMAs at 6 x 32
// instead of 8 x 64 cycles, with fp32-class error (the sum order differs from
// the fp32 MFMA's, as any blocked fp32 GEMM's does).
typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma_bf16(s16x8 a, s16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(__attribute__((ext_vector_type(8))) __bf16, a),
                                                   __builtin_bit_cast(__attribute__((ext_vector_type(8))) __bf16, b),
                                                   c, 0, 0, 0);
}
struct Pieces {
    s16x8 hi, mid, lo;
};
// (x0, x1) → the three piece pairs, element x0 in the low half of each dword
__device__ __forceinline__ void split3(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    h = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{x0, x1}, b2));
    float r0 = x0 - __builtin_bit_cast(float, h << 16), r1 = x1 - __builtin_bit_cast(float, h & 0xffff0000u);
    m = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{r0, r1}, b2));
    r0 -= __builtin_bit_cast(float, m << 16);
    r1 -= __builtin_bit_cast(float, m & 0xffff0000u);
    l = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{r0, r1}, b2));
}
__device__ __forceinline__ Pieces split8(const float (&x)[8]) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t a, b, c;
        split3(x[2 * j], x[2 * j + 1], a, b, c);
        h[j] = a; m[j] = b; l[j] = c;
    }
    return Pieces{__builtin_bit_cast(s16x8, h), __builtin_bit_cast(s16x8, m), __builtin_bit_cast(s16x8, l)};
}
// acc += A·B over one 16-deep k-block, small products first
__device__ __forceinline__ f32x16 mfma3(const Pieces& a, const Pieces& b, f32x16 c) {
    c = mfma_bf16(a.lo, b.hi, c);
    c = mfma_bf16(a.hi, b.lo, c);
    c = mfma_bf16(a.mid, b.mid, c);
    c = mfma_bf16(a.mid, b.hi, c);
    c = mfma_bf16(a.hi, b.mid, c);
    return mfma_bf16(a.hi, b.hi, c);
}

}  // namespace fsplit
}  // namespace rt
