// Probe: achievable HBM copy bandwidth vs launch geometry / vector width /
// loads in flight (design input for the gather kernel's ≥70%-of-peak target).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ a, u32x4* __restrict__ b, long n) {
    const long stride = (long)gridDim.x * 256;
    for (long i0 = (long)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = i0 + u * stride;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = i0 + u * stride;
            if (i < n) { if (NT) __builtin_nontemporal_store(v[u], b + i); else b[i] = v[u]; }
        }
    }
}

template <int U, bool NT>
float run(const u32x4* a, u32x4* b, long n, int grid) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((copy_kernel<U, NT>), dim3(grid), dim3(256), 0, 0, a, b, n);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((copy_kernel<U, NT>), dim3(grid), dim3(256), 0, 0, a, b, n);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return 2.0f * n * 16 / (ms / 10) / 1e6;  // GB/s
}

int main() {
    const long bytes = 4L << 30;  // 4 GiB each way
    const long n = bytes / 16;
    u32x4 *a, *b;
    (void)hipMalloc(&a, bytes); (void)hipMalloc(&b, bytes);
    (void)hipMemset(a, 1, bytes); (void)hipMemset(b, 0, bytes);
    for (int grid : {1024, 2048, 4096, 8192, 16384, 65536}) {
        printf("grid %6d: U1 %6.0f  U4 %6.0f  U8 %6.0f  U4nt %6.0f  U8nt %6.0f GB/s\n", grid,
               run<1, false>(a, b, n, grid), run<4, false>(a, b, n, grid), run<8, false>(a, b, n, grid),
               run<4, true>(a, b, n, grid), run<8, true>(a, b, n, grid));
    }
    return 0;
}
