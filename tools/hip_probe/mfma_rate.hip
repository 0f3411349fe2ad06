// Probe: sustained v_mfma_f32_32x32x2_f32 rate on this box (register operands,
// no memory traffic in the loop), for 1..4 waves per SIMD, to separate the
// fp32 MFMA ceiling from the tower kernels' own overheads.
// Build: hipcc -O3 --offload-arch=gfx950 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a0) {
    f32x16 acc = {};
    float a = a0 + threadIdx.x * 1e-6f, b = a0 - threadIdx.x * 1e-6f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[r];
    if (s == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = s;  // keep the loop alive
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096 * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 64;  // 1024 MFMAs per wave
    for (int blocks_per_cu : {1, 2, 3, 4}) {
        const int blocks = 256 * blocks_per_cu;
        hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double fl = 10.0 * blocks * 4 * iters * 16 * 32.0 * 32 * 2 * 2;
        printf("waves/SIMD %d: %.3f ms per launch, %.1f TF/s (MFMA-only)\n", blocks_per_cu, ms / 10,
               fl / (ms * 1e-3) / 1e12);
    }
    return 0;
}
