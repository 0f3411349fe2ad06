// Fused optimiser step on the flat parameter slab:
// torch.nn.utils.clip_grad_norm_(params, 1.0) + torch.optim.Adam(lr, weight_decay)
// (src/training/trainers/two_tower.py:60-64, 144). Two launches per step
// instead of one clip + ~36 per-tensor Adam updates.
#include "rt_common.h"

namespace rt {
namespace optim {

#ifndef RT_NORM_CHUNK
#define RT_NORM_CHUNK 1024
#endif
// elements per block and pass in the norm pass: 4 per thread, all loads in
// flight together (4096 left 16 per thread behind one another: ~3 us more per step)
constexpr int kChunk = RT_NORM_CHUNK;

__global__ __launch_bounds__(256) void grad_sqnorm_kernel(const float* __restrict__ g,
                                                          const int64_t* __restrict__ offsets,
                                                          double* __restrict__ out, int32_t* step_counter,
                                                          int64_t* seed_counter) {
    __shared__ double red[4];
    const int t = blockIdx.y;
    if (blockIdx.x == 0 && t == 0 && threadIdx.x == 0) {
        if (step_counter) *step_counter += 1;
        if (seed_counter) *seed_counter += 1;
    }
    const int64_t lo = offsets[t], hi = offsets[t + 1];
    if (lo + static_cast<int64_t>(blockIdx.x) * kChunk >= hi) return;  // uniform per block
    double s = 0.0;
    for (int64_t c0 = lo + static_cast<int64_t>(blockIdx.x) * kChunk; c0 < hi;
         c0 += static_cast<int64_t>(gridDim.x) * kChunk) {
        const int64_t c1 = (c0 + kChunk) < hi ? (c0 + kChunk) : hi;
#pragma unroll 4
        for (int64_t e = c0 + threadIdx.x; e < c1; e += 256) {
            const double v = g[e];
            s += v * v;
        }
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&out[t], red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void clip_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        const double* __restrict__ sumsq, int n_tensors,
                                                        float max_norm, float lr, const float* lr_dev, float b1,
                                                        float b2, float eps, float wd, int step,
                                                        const int32_t* step_dev, double* __restrict__ zbuf,
                                                        int64_t zwords) {
    __shared__ float coef_s, step_size_s, bc2_sqrt_s;
    // this thread's first element is loaded before the clip factor is known
    // (it does not depend on it): the two memory round trips overlap
    const int64_t e0 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    float p0 = 0.f, g0 = 0.f, m0 = 0.f, v0 = 0.f;
    if (e0 < n) { p0 = p[e0]; g0 = g[e0]; m0 = m[e0]; v0 = v[e0]; }
    if (threadIdx.x < 64) {
        // wave 0 sums the per-tensor norms in parallel (a fixed tree: deterministic)
        double tot = 0.0;
        for (int t = threadIdx.x; t < n_tensors; t += 64) tot += sumsq[t];
        tot = wave_sum(tot);
        if (threadIdx.x == 0) {
            const float total = static_cast<float>(sqrt(tot));
            const float coef = max_norm / (total + 1e-6f);
            coef_s = coef < 1.f ? coef : 1.f;
            const int st = step_dev ? *step_dev : step;
            const float lr_v = lr_dev ? *lr_dev : lr;
            const double bc1 = 1.0 - pow(static_cast<double>(b1), st);
            const double bc2 = 1.0 - pow(static_cast<double>(b2), st);
            step_size_s = static_cast<float>(lr_v / bc1);
            bc2_sqrt_s = static_cast<float>(sqrt(bc2));
        }
    }
    __syncthreads();
    const float coef = coef_s, step_size = step_size_s, bc2s = bc2_sqrt_s;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    auto update = [&](int64_t e, float pv, float graw, float mo, float vo) {
        float gv = graw * coef;
        if (wd != 0.f) gv = gv + wd * pv;
        const float mv = mo + (1.f - b1) * (gv - mo);              // exp_avg.lerp_(grad, 1-beta1)
        const float vv = vo * b2 + (1.f - b2) * gv * gv;           // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
        const float denom = sqrtf(vv) / bc2s + eps;
        m[e] = mv;
        v[e] = vv;
        p[e] = pv - step_size * (mv / denom);
        g[e] = 0.f;  // consumed: the next step accumulates from zero
    };
    if (e0 < n) update(e0, p0, g0, m0, v0);
    for (int64_t e = e0 + stride; e < n; e += stride) update(e, p[e], g[e], m[e], v[e]);
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; e < zwords; e += stride) zbuf[e] = 0.0;
}

}  // namespace optim
}  // namespace rt

using namespace rt;

extern "C" int rt_grad_sqnorm(const float* grads, const int64_t* offsets, int n_tensors, double* sumsq_out,
                              int32_t* step_counter, int64_t* seed_counter, void* stream) {
    if (n_tensors < 0 || (n_tensors > 0 && (!grads || !offsets || !sumsq_out))) return RT_ERR_INVALID;
    if (n_tensors == 0) return RT_OK;
    // offsets live on the device: 64 blocks per tensor, each striding over chunks;
    // blocks past a small tensor's end exit at once
    const dim3 grid(64, static_cast<unsigned>(n_tensors));
    hipLaunchKernelGGL(optim::grad_sqnorm_kernel, grid, dim3(256), 0, as_stream(stream), grads, offsets, sumsq_out,
                       step_counter, seed_counter);
    return check_launch("grad_sqnorm_kernel");
}

extern "C" int rt_clip_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                                 const double* sumsq, int n_tensors, float max_norm, float lr, const float* lr_dev,
                                 float beta1, float beta2, float eps, float weight_decay, int step,
                                 const int32_t* step_dev, double* zero_buf, int64_t zero_words, void* stream) {
    if (n < 0 || !params || !grads || !exp_avg || !exp_avg_sq || !sumsq || n_tensors <= 0) return RT_ERR_INVALID;
    if (!step_dev && step < 1) return RT_ERR_INVALID;
    if (zero_words < 0 || (zero_words > 0 && !zero_buf)) return RT_ERR_INVALID;
    if (n == 0) return RT_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(optim::clip_adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, as_stream(stream),
                       params, grads, exp_avg, exp_avg_sq, n, sumsq, n_tensors, max_norm, lr, lr_dev, beta1, beta2,
                       eps, weight_decay, step, step_dev, zero_buf, zero_words);
    return check_launch("clip_adam_kernel");
}
