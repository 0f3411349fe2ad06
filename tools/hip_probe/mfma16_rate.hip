// Probe: what bounds the 16-bit top-K scan's MFMA loop (topk_v4.h) without any
// selection. The v4 geometry in miniature: 8 waves per block, one block per CU
// (LDS-limited), 2 waves per SIMD, each wave 2 query sets of 32 (B fragments in
// registers), 128-row LDS stages of 32-row sub-tiles with a one-chunk row pad,
// 8 dependent v_mfma_f32_32x32x16_f16 per set, random operands.
// Variants (MODE bits): 1 = read A fragments from LDS (next sub-tile behind set
// 1's MFMAs), 2 = pin each set's result with an empty asm (as v4 does before its
// store loop), 4 = block barrier every stage, 8 = 16 VALU per set (v_max chain).
// Build: hipcc -O3 --offload-arch=gfx950 mfma16_rate.hip -o mfma16_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int RS = 17 * 16;  // LDS row stride (16 data chunks + pad)
constexpr int NT = 128;

template <int MODE>
__global__ __launch_bounds__(512) void scan(float* out, int stages) {
    __shared__ __attribute__((aligned(16))) char lds[3 * NT * RS];  // 104 KiB: one block per CU
    const int tid = threadIdx.x, lane = tid & 63, col = lane & 31, half = lane >> 5;
    for (int i = tid; i < 3 * NT * RS / 16; i += 512) {
        const unsigned x = (i * 2654435761u) ^ (blockIdx.x * 40503u);
        reinterpret_cast<uint4*>(lds)[i] = make_uint4(x & 0x3bff3bffu, (x >> 3) & 0x3bff3bffu, x & 0x37ff37ffu,
                                                      (x >> 5) & 0x3bff3bffu);
    }
    __syncthreads();
    h8 qf[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 8; ++s)
            for (int e = 0; e < 8; ++e) qf[j][s][e] = static_cast<_Float16>(((lane * 7 + s * 3 + j + e) % 13) * 0.01f);
    const char* base = lds + col * RS + half * 16;
    h8 af[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) af[s] = __builtin_bit_cast(h8, *reinterpret_cast<const uint4*>(base + s * 32));
    float sink = 0.f;
    f32x16 acc0, acc1;
    for (int v = 0; v < stages; ++v) {
        const char* stage = base + (v % 3) * NT * RS;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
            acc0 = f32x16{};
#pragma unroll
            for (int s = 0; s < 8; ++s) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s], qf[0][s], acc0, 0, 0, 0);
            if constexpr (MODE & 2) asm volatile("" : "+v"(acc0));
            if constexpr (MODE & 8) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sink = fmaxf(sink, acc1[r]);
            }
            acc1 = f32x16{};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s], qf[1][s], acc1, 0, 0, 0);
                if constexpr (MODE & 1) {
                    const char* nsrc = rt < 3 ? stage + (rt + 1) * 32 * RS : base + ((v + 1) % 3) * NT * RS;
                    af[s] = __builtin_bit_cast(h8, *reinterpret_cast<const uint4*>(nsrc + s * 32));
                }
            }
            if constexpr (MODE & 2) asm volatile("" : "+v"(acc1));
            if constexpr (MODE & 8) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sink = fmaxf(sink, acc0[r]);
            }
        }
        if constexpr (MODE & 4) __syncthreads();
    }
    float s = sink;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
    if (s == 12345.f) out[blockIdx.x * 512 + tid] = s;
}

template <int MODE>
void run(float* out, int stages) {
    hipLaunchKernelGGL(scan<MODE>, dim3(256), dim3(512), 0, 0, out, stages);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(scan<MODE>, dim3(256), dim3(512), 0, 0, out, stages);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl = 5.0 * 256 * 8 * stages * 4 * 2 * 8 * (2.0 * 32 * 32 * 16);
    printf("mode %2d (lds %d pin %d barrier %d valu %d): %.3f ms  %.0f TF/s  %.1f%% of 2.5 PF\n", MODE, MODE & 1,
           (MODE >> 1) & 1, (MODE >> 2) & 1, (MODE >> 3) & 1, ms / 5, fl / (ms * 1e-3) / 1e12,
           fl / (ms * 1e-3) / 1e12 / 25.0);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 512 * 4);
    const int stages = 2000;
    run<0>(out, stages);
    run<1>(out, stages);
    run<2>(out, stages);
    run<3>(out, stages);
    run<5>(out, stages);
    run<7>(out, stages);
    run<13>(out, stages);
    run<15>(out, stages);
    run<9>(out, stages);
    return 0;
}
