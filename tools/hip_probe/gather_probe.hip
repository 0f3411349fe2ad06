// Row-gather bandwidth probe (C5 shard shape: 12.5M x 512-B rows, 16M random
// ids): variants of in-flight depth, cache policy and lane mapping.
// Build: hipcc -O3 --offload-arch=gfx950 gather_probe.hip -o gather_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT_LOAD, bool NT_STORE>
__global__ __launch_bounds__(256) void gather_flat(const u32x4* __restrict__ t, const int64_t* __restrict__ ids,
                                                   int64_t n_ids, u32x4* __restrict__ out) {
    const uint32_t vpr = 32;  // 512-B rows
    const uint32_t total = static_cast<uint32_t>(n_ids) * vpr;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += stride * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * stride;
            if (e < total) {
                const int64_t id = ids[e >> 5];
                const u32x4* src = t + id * vpr + (e & 31);
                v[u] = NT_LOAD ? __builtin_nontemporal_load(src) : *src;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * stride;
            if (e < total) {
                if (NT_STORE) __builtin_nontemporal_store(v[u], out + e);
                else out[e] = v[u];
            }
        }
    }
}

// one wave per group of R rows: lane l copies chunk (l & 31) of row (l >> 5) + 2k
template <int R>
__global__ __launch_bounds__(256) void gather_rowwave(const u32x4* __restrict__ t, const int64_t* __restrict__ ids,
                                                      int64_t n_ids, u32x4* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    for (int64_t r0 = wave * R; r0 < n_ids; r0 += nw * R) {
        u32x4 v[R / 2];
        int64_t id[R / 2];
#pragma unroll
        for (int k = 0; k < R / 2; ++k) {
            const int64_t r = r0 + 2 * k + (lane >> 5);
            id[k] = r < n_ids ? ids[r] : -1;
        }
#pragma unroll
        for (int k = 0; k < R / 2; ++k)
            if (id[k] >= 0) v[k] = __builtin_nontemporal_load(t + id[k] * 32 + (lane & 31));
#pragma unroll
        for (int k = 0; k < R / 2; ++k) {
            const int64_t r = r0 + 2 * k + (lane >> 5);
            if (r < n_ids) __builtin_nontemporal_store(v[k], out + r * 32 + (lane & 31));
        }
    }
}

__global__ void read_only(const u32x4* __restrict__ t, const int64_t* __restrict__ ids, int64_t n_ids,
                          unsigned* sink) {
    const uint32_t total = static_cast<uint32_t>(n_ids) * 32;
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (uint32_t e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += stride * 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t e = e0 + u * stride;
            v[u] = e < total ? __builtin_nontemporal_load(t + ids[e >> 5] * 32 + (e & 31)) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int64_t rows = 12500000, n = 16777216;
    u32x4 *t, *o;
    int64_t* ids;
    unsigned* sink;
    hipMalloc(&t, rows * 512);
    hipMalloc(&o, n * 512);
    hipMalloc(&ids, n * 8);
    hipMalloc(&sink, 4);
    hipMemset(t, 1, rows * 512);
    std::vector<int64_t> h(n);
    std::mt19937_64 rng(1);
    for (auto& x : h) x = rng() % rows;
    hipMemcpy(ids, h.data(), n * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto launch, double bytes) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("%-36s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    const double rw = 2.0 * n * 512 + 8.0 * n;
    for (int rep = 0; rep < 2; ++rep) {
        run("flat U1 nt/nt grid 2097152", [&] { gather_flat<1, true, true><<<2097152, 256>>>(t, ids, n, o); }, rw);
        run("flat U1 nt/nt grid 1048576 (2 it)", [&] { gather_flat<1, true, true><<<1048576, 256>>>(t, ids, n, o); }, rw);
        run("flat U2 nt/nt grid 524288", [&] { gather_flat<2, true, true><<<524288, 256>>>(t, ids, n, o); }, rw);
        run("flat U4 nt/nt grid 262144", [&] { gather_flat<4, true, true><<<262144, 256>>>(t, ids, n, o); }, rw);
        run("flat U1 plain/nt grid 2097152", [&] { gather_flat<1, false, true><<<2097152, 256>>>(t, ids, n, o); }, rw);
        run("flat U4 nt/nt grid 65536 (current)", [&] { gather_flat<4, true, true><<<65536, 256>>>(t, ids, n, o); }, rw);
    }
    run("read only (bytes = reads)", [&] { read_only<<<65536, 256>>>(t, ids, n, sink); }, 1.0 * n * 512 + 8.0 * n);
    run("hipMemcpy d2d 8 GB", [&] { hipMemcpyAsync(o, t, rows * 512, hipMemcpyDeviceToDevice); }, 2.0 * rows * 512);
    return 0;
}
