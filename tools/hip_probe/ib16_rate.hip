// Probe: the MFMA issue rate of the C5 in-batch gradient pass (inbatch16.hip ROW
// / COL) without memory: 4 waves per block (one per SIMD, 512-register file),
// per 32-row sub-tile 16 dependent S MFMAs (v_mfma_f32_32x32x16_bf16, B operand
// resident) and 32 gradient MFMAs into 8 accumulator tiles (hi, lo per d block
// and k half), the dS operand derived from the S accumulator by VALU.
// MODE: 0 = S + gradient (the pass), 1 = S chain only, 2 = gradient only,
//       3 = the pass with the gradient MFMAs interleaved over d blocks
// Build: hipcc -O3 --offload-arch=gfx950 ib16_rate.hip -o ib16_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

__device__ inline b8 mk(int seed, int lane) {
    b8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = static_cast<__bf16>(((lane * 7 + seed * 3 + e) % 13) * 0.01f);
    return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void pass(float* out, int iters) {
    const int lane = threadIdx.x & 63;
    b8 qf[16], af[16], ga[8][2];
#pragma unroll
    for (int s = 0; s < 16; ++s) { qf[s] = mk(s, lane); af[s] = mk(s + 16, lane); }
#pragma unroll
    for (int d = 0; d < 8; ++d) { ga[d][0] = mk(d + 40, lane); ga[d][1] = mk(d + 50, lane); }
    f32x16 gacc[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) gacc[d] = f32x16{};
    f32x16 acc = {};
    for (int it = 0; it < iters; ++it) {
        f32x16 accn = {};
        if constexpr (MODE != 2) {
#pragma unroll
            for (int s = 0; s < 16; ++s) accn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], qf[s], accn, 0, 0, 0);
        }
        if constexpr (MODE != 1) {
            b8 bh[2], bl[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2 x{acc[8 * s2 + 2 * j] * 0.01f, acc[8 * s2 + 2 * j + 1] * 0.01f};
                    const b2 hv = __builtin_convertvector(x, b2);
                    const f32x2 r{x[0] - static_cast<float>(hv[0]), x[1] - static_cast<float>(hv[1])};
                    const b2 lv = __builtin_convertvector(r, b2);
                    bh[s2][2 * j] = hv[0]; bh[s2][2 * j + 1] = hv[1];
                    bl[s2][2 * j] = lv[0]; bl[s2][2 * j + 1] = lv[1];
                }
            if constexpr (MODE == 3) {
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int hl = 0; hl < 2; ++hl)
#pragma unroll
                        for (int d = 0; d < 8; ++d)
                            gacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[d][s2], hl ? bl[s2] : bh[s2], gacc[d], 0, 0, 0);
            } else {
#pragma unroll
                for (int d = 0; d < 8; ++d)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        gacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[d][s2], bh[s2], gacc[d], 0, 0, 0);
                        gacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[d][s2], bl[s2], gacc[d], 0, 0, 0);
                    }
            }
        }
        acc = MODE == 2 ? acc + 1.f : accn;
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        s += acc[r];
#pragma unroll
        for (int d = 0; d < 8; ++d) s += gacc[d][r];
    }
    if (s == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(float* out, int iters) {
    hipLaunchKernelGGL(pass<MODE>, dim3(256), dim3(256), 0, 0, out, iters);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(pass<MODE>, dim3(256), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const int per = MODE == 1 ? 16 : MODE == 2 ? 32 : 48;
    const double mfma_per_simd = static_cast<double>(iters) * per;  // one wave per SIMD, one block per CU
    const double ns = ms / 5 * 1e6;
    printf("mode %d: %.3f ms  %.2f ns per MFMA per SIMD (= %.1f cycles at 2.4 GHz)  %.1f%% of 2.5 PF\n", MODE, ms / 5,
           ns / mfma_per_simd, ns / mfma_per_simd * 2.4, 100.0 * 32.0 / (ns / mfma_per_simd * 2.4));
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 256 * 4);
    const int iters = 4000;
    run<0>(out, iters);
    run<1>(out, iters);
    run<2>(out, iters);
    run<3>(out, iters);
    run<0>(out, iters);
    return 0;
}
