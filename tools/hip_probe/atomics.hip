// Probe: cost of global atomics vs contention on gfx950 (design input for the
// split-M dW reduction and the BatchNorm column-stat accumulation).
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void atom_kernel(T* dst, int n_addr, int per_block) {
    // block b adds per_block values to addresses [(b*per_block + i) % n_addr]
    for (int i = threadIdx.x; i < per_block; i += blockDim.x) {
        const int a = (blockIdx.x * per_block + i) % n_addr;
        atomicAdd(&dst[a], static_cast<T>(1));
    }
}
__global__ void store_kernel(float* dst, int n_addr, int per_block) {
    for (int i = threadIdx.x; i < per_block; i += blockDim.x)
        dst[(static_cast<long>(blockIdx.x) * per_block + i)] = 1.f;
}

template <typename T>
float run(int blocks, int per_block, int n_addr) {
    T* d; hipMalloc(&d, sizeof(T) * (size_t)n_addr);
    hipMemset(d, 0, sizeof(T) * (size_t)n_addr);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) atom_kernel<T><<<blocks, 256>>>(d, n_addr, per_block);
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) atom_kernel<T><<<blocks, 256>>>(d, n_addr, per_block);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipFree(d);
    return ms / 20 * 1000.f;
}

int main() {
    printf("%-8s %8s %8s %8s %10s %8s\n", "type", "blocks", "perblk", "naddr", "us", "Gatom/s");
    struct C { int blocks, per, naddr; } cs[] = {
        {512, 256, 256}, {512, 256, 256 * 16}, {512, 512, 512}, {512, 512, 512 * 16},
        {512, 4096, 32768}, {64, 32768, 32768}, {128, 32768, 32768}, {8, 32768, 32768}, {512, 128, 128}};
    for (auto c : cs) {
        float us = run<double>(c.blocks, c.per, c.naddr);
        printf("%-8s %8d %8d %8d %10.2f %8.2f\n", "f64", c.blocks, c.per, c.naddr, us, c.blocks * (double)c.per / us / 1e3);
        us = run<float>(c.blocks, c.per, c.naddr);
        printf("%-8s %8d %8d %8d %10.2f %8.2f\n", "f32", c.blocks, c.per, c.naddr, us, c.blocks * (double)c.per / us / 1e3);
    }
    // empty-ish kernel baseline (launch + 512 blocks storing 256 floats)
    float* d; hipMalloc(&d, 512 * 256 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) store_kernel<<<512, 256>>>(d, 0, 256);
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) store_kernel<<<512, 256>>>(d, 0, 256);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("store baseline 512x256: %.2f us/launch\n", ms / 20 * 1000.f);
    return 0;
}
