// Probe: split-M dW kernel variants (atomics vs partial stores, split count,
// prologue mode) on the C2 negative-tower shape. Includes the library source.
#include "../../real-time-recommendation-system-with-feature-store_amd/csrc/mlp.hip"
#include <cstdio>
#include <vector>

template <typename F>
static float time_us(F f, int reps = 30) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps * 1000.f;
}

__global__ void copy_kernel(const float4* a, float4* b, int64_t n) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

int main() {
    struct Shape { int64_t m; int k, n; } shapes[] = {{16384, 256, 128}, {16384, 20, 256}, {16384, 128, 128}, {1024, 256, 128}};
    for (auto sh : shapes) {
        const int64_t m = sh.m; const int k = sh.k, n = sh.n;
        float *src, *dz, *dw, *db, *g, *b, *mean, *inv;
        (void)hipMalloc(&src, m * k * 4); (void)hipMalloc(&dz, m * n * 4);
        (void)hipMalloc(&dw, 64LL * n * k * 4); (void)hipMalloc(&db, n * 4);
        (void)hipMalloc(&g, k * 4); (void)hipMalloc(&b, k * 4); (void)hipMalloc(&mean, k * 4); (void)hipMalloc(&inv, k * 4);
        (void)hipMemset(src, 0, m * k * 4); (void)hipMemset(dz, 0, m * n * 4);
        (void)hipMemset(g, 0, k * 4); (void)hipMemset(b, 0, k * 4); (void)hipMemset(mean, 0, k * 4); (void)hipMemset(inv, 0, k * 4);
        for (int mode : {0, 1}) {
            for (int splits : {8, 16, 32, 64}) {
                rt_linear_bwd_args a{};
                a.m = m; a.k = k; a.n = n; a.dw = dw; a.dbias = db; a.dz_ws = dz; a.src = src; a.src_rows = m; a.ld_src = k;
                a.prev_mode = mode; a.prev_act = 0;
                if (mode == 1) { a.prev_mean = mean; a.prev_invstd = inv; a.prev_gamma = g; a.prev_beta = b; a.prev_drop_p = 0.2f; a.prev_drop_seed = 7; }
                const int kt = k <= 32 ? 1 : 2;
                const int tn = (n + 63) / 64, tk = (k + 32 * kt - 1) / (32 * kt);
                int64_t rps = (m + splits - 1) / splits; rps = (rps + 63) / 64 * 64;
                const int64_t sp = (m + rps - 1) / rps;
                dim3 grid(tn, tk, sp);
                float ta;
                if (kt == 1) {
                    if (mode == 0) ta = time_us([&] { hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<1, 0>), grid, dim3(256), 0, 0, a, rps); });
                    else ta = time_us([&] { hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<1, 2>), grid, dim3(256), 0, 0, a, rps); });
                } else {
                    if (mode == 0) ta = time_us([&] { hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<2, 0>), grid, dim3(256), 0, 0, a, rps); });
                    else ta = time_us([&] { hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<2, 2>), grid, dim3(256), 0, 0, a, rps); });
                }
                printf("m=%6lld k=%3d n=%3d pro=%d splits=%2lld blocks=%4lld  %7.1f us  (%.1f TF/s)\n",
                       (long long)m, k, n, mode ? 2 : 0, (long long)sp, (long long)(tn * tk * sp), ta, 2.0 * m * n * k / ta / 1e6);
            }
        }
        const int64_t nv = (m * k) / 4;
        float tc = time_us([&] { hipLaunchKernelGGL(copy_kernel, dim3(1024), dim3(256), 0, 0, (const float4*)src, (float4*)dz, nv < m * n / 4 ? nv : m * n / 4); });
        printf("  copy of min(src,dz) bytes: %.1f us\n", tc);
        (void)hipFree(src); (void)hipFree(dz); (void)hipFree(dw); (void)hipFree(db);
        (void)hipFree(g); (void)hipFree(b); (void)hipFree(mean); (void)hipFree(inv);
    }
    return 0;
}
