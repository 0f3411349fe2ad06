// Two-tower losses, fused forward + backward (fp32 scores on v_mfma_f32_32x32x2_f32).
//
// Replaces (src/models/two_tower.py):
//   compute_similarity      :380-404   → rt_similarity_f32
//   contrastive_loss        :406-451   (explicit negatives, biases on the positive logit only)
//   in_batch_negative_loss  :453-479   (S = U·Pᵀ/τ, CE with diagonal labels)
// and the trainer's mixing 0.7·explicit + 0.3·in-batch
// (src/training/trainers/two_tower.py:111-137), forward AND backward.
//
// Launch 1 (one block per 32 users): explicit CE with its gradients, then the
//   in-batch row log-sum-exp by streaming 32-row item tiles through MFMA with an
//   online max/sum (S never stored).
// Launch 2 (2 × B/32 blocks): S is recomputed tile by tile; row blocks
//   accumulate dU = dS·P, column blocks dP = dSᵀ·U (dS = w/B·(softmax(S) − I)),
//   each wave owning a 32-wide slice of the tiles, reduced through LDS.
// The k-order inside an MFMA chain is permuted (k = h·D/2 + s) so that every
// fragment load is a contiguous 16-byte vector.
#include <float.h>

#include "rt_common.h"

namespace rt {
namespace loss {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int RB = 32;        // users (or items) per block
constexpr int kMaxD = 256;
constexpr int kMaxNeg = 64;
constexpr int NG = 16;  // negatives reduced together

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// acc[r] = <A[a0 + tile_row(r,h)], Bm[b0 + (lane&31)]> (raw dot products)
__device__ __forceinline__ f32x16 dot_tile(const float* __restrict__ A, int64_t a0, int64_t na,
                                           const float* __restrict__ Bm, int64_t b0, int64_t nb, int D) {
    const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    int64_t ar = a0 + c, br = b0 + c;
    ar = ar < na ? ar : na - 1;
    br = br < nb ? br : nb - 1;
    const float* pa = A + ar * D + h * (D / 2);
    const float* pb = Bm + br * D + h * (D / 2);
    f32x16 acc = {};
    int s = 0;
    for (; s + 16 <= D / 2; s += 16) {  // 8 independent 16-byte loads in flight
        float4 av[4], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            av[j] = *reinterpret_cast<const float4*>(pa + s + 4 * j);
            bv[j] = *reinterpret_cast<const float4*>(pb + s + 4 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc = mfma(av[j].x, bv[j].x, acc);
            acc = mfma(av[j].y, bv[j].y, acc);
            acc = mfma(av[j].z, bv[j].z, acc);
            acc = mfma(av[j].w, bv[j].w, acc);
        }
    }
    for (; s < D / 2; s += 4) {
        const float4 av = *reinterpret_cast<const float4*>(pa + s);
        const float4 bv = *reinterpret_cast<const float4*>(pb + s);
        acc = mfma(av.x, bv.x, acc);
        acc = mfma(av.y, bv.y, acc);
        acc = mfma(av.z, bv.z, acc);
        acc = mfma(av.w, bv.w, acc);
    }
    return acc;
}

struct Args {
    const float* u; const float* p; const float* q;
    int64_t b; int d; int n_neg; float inv_tau;
    const float* ub; const float* ib;
    float we, wb;       // weights of the explicit / in-batch terms in loss_out[0]
    double* loss;
    float* du; float* dp; float* dq; float* dub; float* dib;
    float2* part;       // workspace [n_split][b]: per-split (max, sum exp) of S rows
    float* diag;        // workspace [b]: S_ii = u_i·p_i / tau
    int n_split;        // item splits of 128 (JT) per user tile
    bool grad;
};

constexpr int JT = 128;  // streamed rows per block (4 waves x 32)

// ---------------------------------------------------------------- launch 1
// block (it, js): in-batch partial row log-sum-exp of users [32it, 32it+32) over
// items [128js, 128js+128) (one 32x32 S^T tile per wave), plus the explicit
// contrastive CE of a strided subset of the tile's users (one wave per user).
__global__ __launch_bounds__(256) void loss_fwd_kernel(Args a) {
    __shared__ float negs[4][kMaxNeg];
    __shared__ float red_m[4][RB], red_l[4][RB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int it = blockIdx.x, js = blockIdx.y;
    const int64_t i0 = static_cast<int64_t>(it) * RB;
    const int D = a.d;
    const float bias = (a.ub ? a.ub[0] : 0.f) + (a.ib ? a.ib[0] : 0.f);
    const float inv_b = 1.f / static_cast<float>(a.b);

    // ---- in-batch partial lse: S^T tile (items j × users i) ----
    {
        const int64_t t = static_cast<int64_t>(js) * 4 + w;   // item tile of this wave
        float om = -INFINITY, ol = 0.f;
        if (t * 32 < a.b) {
            const f32x16 acc = dot_tile(a.p, t * 32, a.b, a.u, i0, a.b, D);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t j = t * 32 + tile_row(r, h);
                if (j < a.b) {
                    const float sv = acc[r] * a.inv_tau;
                    if (sv > om) { ol = ol * expf(om - sv) + 1.f; om = sv; }
                    else ol += expf(sv - om);
                }
            }
        }
        const float m2 = __shfl_xor(om, 32, 64), l2 = __shfl_xor(ol, 32, 64);
        const float mm = fmaxf(om, m2);
        ol = (mm == -INFINITY) ? 0.f : ol * expf(om - mm) + l2 * expf(m2 - mm);
        if (h == 0) { red_m[w][c] = mm; red_l[w][c] = ol; }
    }
    __syncthreads();
    if (w == 0 && h == 0 && i0 + c < a.b) {
        float mm = -INFINITY;
        for (int x = 0; x < 4; ++x) mm = fmaxf(mm, red_m[x][c]);
        float ll = 0.f;
        if (mm != -INFINITY)
            for (int x = 0; x < 4; ++x) ll += red_l[x][c] * expf(red_m[x][c] - mm);
        a.part[static_cast<int64_t>(js) * a.b + i0 + c] = make_float2(mm, ll);
    }

    // ---- explicit negatives: users ii = 4js + w, stepping 4*n_split ----
    double loss_e = 0.0;
    float dbias_acc = 0.f;
    for (int ii = js * 4 + w; ii < RB; ii += 4 * a.n_split) {
        const int64_t i = i0 + ii;
        if (i >= a.b) break;
        const float* ur = a.u + i * D;
        const float* pr = a.p + i * D;
        float uv[kMaxD / 64], pv[kMaxD / 64];
        float part = 0.f;
#pragma unroll
        for (int t = 0; t < kMaxD / 64; ++t) {
            const int dd = lane + 64 * t;
            uv[t] = dd < D ? ur[dd] : 0.f;
            pv[t] = dd < D ? pr[dd] : 0.f;
            part += uv[t] * pv[t];
        }
        const float dup = wave_sum(part) * a.inv_tau;
        if (lane == 0) a.diag[i] = dup;
        if (a.n_neg <= 0) {
            if (a.grad) {
#pragma unroll
                for (int t = 0; t < kMaxD / 64; ++t) {
                    const int dd = lane + 64 * t;
                    if (dd < D) { a.du[i * D + dd] = 0.f; a.dp[i * D + dd] = 0.f; }
                }
            }
            continue;
        }
        const float pos = dup + bias;
        // all negative dots of a group of 16 at once: independent loads, one
        // butterfly reduction for the 16 partial sums
        float mx = pos;
        for (int g0 = 0; g0 < a.n_neg; g0 += NG) {
            float part_j[NG];
#pragma unroll
            for (int jj = 0; jj < NG; ++jj) {
                part_j[jj] = 0.f;
                const int j = g0 + jj;
                if (j < a.n_neg) {
                    const float* qr = a.q + (i * a.n_neg + j) * D;
#pragma unroll
                    for (int t = 0; t < kMaxD / 64; ++t) {
                        const int dd = lane + 64 * t;
                        if (dd < D) part_j[jj] += uv[t] * qr[dd];
                    }
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
#pragma unroll
                for (int jj = 0; jj < NG; ++jj) part_j[jj] += __shfl_xor(part_j[jj], o, 64);
#pragma unroll
            for (int jj = 0; jj < NG; ++jj) {
                if (g0 + jj < a.n_neg) {
                    const float nv = part_j[jj] * a.inv_tau;
                    if (lane == 0) negs[w][g0 + jj] = nv;
                    mx = fmaxf(mx, nv);
                }
            }
        }
        wave_lds_sync();
        float se = expf(pos - mx);
        for (int j = 0; j < a.n_neg; ++j) se += expf(negs[w][j] - mx);
        const float lse = mx + logf(se);
        if (lane == 0) loss_e += static_cast<double>(lse - pos);
        if (a.grad) {
            const float dpos = a.we * inv_b * (expf(pos - lse) - 1.f);
            if (lane == 0) dbias_acc += dpos;
            float duv[kMaxD / 64];
#pragma unroll
            for (int t = 0; t < kMaxD / 64; ++t) duv[t] = dpos * pv[t];
            for (int g0 = 0; g0 < a.n_neg; g0 += NG) {
                float qv[NG][kMaxD / 64];
#pragma unroll
                for (int jj = 0; jj < NG; ++jj) {
                    const int j = g0 + jj;
                    const float* qr = a.q + (i * a.n_neg + (j < a.n_neg ? j : 0)) * D;
#pragma unroll
                    for (int t = 0; t < kMaxD / 64; ++t) {
                        const int dd = lane + 64 * t;
                        qv[jj][t] = (j < a.n_neg && dd < D) ? qr[dd] : 0.f;
                    }
                }
#pragma unroll
                for (int jj = 0; jj < NG; ++jj) {
                    const int j = g0 + jj;
                    if (j >= a.n_neg) break;
                    const float dn = a.we * inv_b * expf(negs[w][j] - lse);
                    float* dqr = a.dq + (i * a.n_neg + j) * D;
#pragma unroll
                    for (int t = 0; t < kMaxD / 64; ++t) {
                        const int dd = lane + 64 * t;
                        if (dd < D) {
                            duv[t] += dn * qv[jj][t];
                            dqr[dd] = dn * uv[t] * a.inv_tau;
                        }
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < kMaxD / 64; ++t) {
                const int dd = lane + 64 * t;
                if (dd < D) {
                    a.du[i * D + dd] = duv[t] * a.inv_tau;
                    a.dp[i * D + dd] = dpos * uv[t] * a.inv_tau;
                }
            }
        }
        wave_lds_sync();
    }
    if (lane == 0 && loss_e != 0.0) {
        const double le = loss_e / static_cast<double>(a.b);
        atomicAdd(&a.loss[1], le);
        atomicAdd(&a.loss[0], a.we * le);
    }
    if (lane == 0 && a.grad && a.n_neg > 0 && dbias_acc != 0.f) {
        if (a.dub) atomicAdd(a.dub, dbias_acc);
        if (a.dib) atomicAdd(a.dib, dbias_acc);
    }
}

// combine the per-split partials of user i into its log-sum-exp
__device__ __forceinline__ float combine_lse(const float2* part, int n_split, int64_t b, int64_t i) {
    float mm = -INFINITY;
    for (int s = 0; s < n_split; ++s) mm = fmaxf(mm, part[static_cast<int64_t>(s) * b + i].x);
    float ll = 0.f;
    for (int s = 0; s < n_split; ++s) {
        const float2 v = part[static_cast<int64_t>(s) * b + i];
        if (v.x != -INFINITY) ll += v.y * expf(v.x - mm);
    }
    return mm + logf(ll);
}

// ---------------------------------------------------------------- launch 2
// blockIdx.z = 0: row pass, fixed 32 users, dU += dS · P over 128 streamed items
// blockIdx.z = 1: column pass, fixed 32 items, dP += dSᵀ · U over 128 streamed users
// (dS = wb/B·(softmax(S) − I)); results added atomically (n_split adds per element).
template <int DT>  // D/32 output tiles per wave accumulator
__global__ __launch_bounds__(256) void loss_bwd_kernel(Args a, float wb_eff, bool add_loss) {
    __shared__ float Ds[4][32][33];
    __shared__ float lse_s[JT];       // row pass: [0,32) fixed users; column pass: 128 streamed users
    __shared__ float red[32 * (kMaxD + 1)];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int D = a.d;
    const bool row_pass = blockIdx.z == 0;
    const int64_t f0 = static_cast<int64_t>(blockIdx.x) * RB;      // fixed tile
    const int64_t s0 = static_cast<int64_t>(blockIdx.y) * JT;      // streamed range
    const float* Str = row_pass ? a.p : a.u;
    const float scale = wb_eff / static_cast<float>(a.b);
    if (row_pass) {
        if (tid < RB) {
            const int64_t i = f0 + tid;
            const float l = i < a.b ? combine_lse(a.part, a.n_split, a.b, i) : 0.f;
            lse_s[tid] = l;
            if (add_loss && blockIdx.y == 0 && i < a.b) {
                const double li = static_cast<double>(l - a.diag[i]) / static_cast<double>(a.b);
                atomicAdd(&a.loss[2], li);
                atomicAdd(&a.loss[0], static_cast<double>(wb_eff) * li);
            }
        }
    } else if (tid < JT) {
        const int64_t i = s0 + tid;
        lse_s[tid] = i < a.b ? combine_lse(a.part, a.n_split, a.b, i) : 0.f;
    }
    for (int e = tid; e < 32 * (kMaxD + 1); e += 256) red[e] = 0.f;
    __syncthreads();
    if (!a.grad) return;
    f32x16 acc[DT];
#pragma unroll
    for (int x = 0; x < DT; ++x) acc[x] = f32x16{};
    const int64_t t0 = s0 + w * 32;  // this wave's streamed tile
    if (t0 < a.b) {
        // row pass: (row = item j, col = user i);  column pass: (row = user i, col = item j)
        const f32x16 st = row_pass ? dot_tile(a.p, t0, a.b, a.u, f0, a.b, D)
                                   : dot_tile(a.u, t0, a.b, a.p, f0, a.b, D);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rr = tile_row(r, h);
            const int64_t srow = t0 + rr;
            const int64_t fcol = f0 + c;
            float ds = 0.f;
            if (srow < a.b && fcol < a.b) {
                const float lse = row_pass ? lse_s[c] : lse_s[w * 32 + rr];
                const float pr = expf(st[r] * a.inv_tau - lse);
                ds = scale * (pr - (srow == fcol ? 1.f : 0.f));
            }
            Ds[w][c][rr] = ds;  // [fixed][streamed]
        }
        wave_lds_sync();
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            const int dcol = dt * 32 + c;
#pragma unroll 4
            for (int s = 0; s < 16; ++s) {
                const int ks = 2 * s + h;
                const int64_t sr = t0 + ks;
                const float bv = (sr < a.b && dcol < D) ? Str[sr * D + dcol] : 0.f;
                acc[dt] = mfma(Ds[w][c][ks], bv, acc[dt]);
            }
        }
    }
    // reduce the 4 wave partials through LDS (red[fixed][d]), then atomically add
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) atomicAdd(&red[tile_row(r, h) * (kMaxD + 1) + dt * 32 + c], acc[dt][r]);
    __syncthreads();
    float* out = row_pass ? a.du : a.dp;
    for (int e = tid; e < 32 * D; e += 256) {
        const int f = e / D, dd = e % D;
        const int64_t gi = f0 + f;
        if (gi < a.b) atomicAdd(&out[gi * D + dd], red[f * (kMaxD + 1) + dd] * a.inv_tau);
    }
}

// ---------------------------------------------------------------- similarity
__global__ __launch_bounds__(256) void similarity_kernel(const float* u, const float* v, int64_t b, int d,
                                                         float inv_tau, const float* ub, const float* ib,
                                                         float* out) {
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (i >= b) return;
    float s = 0.f;
    for (int dd = lane; dd < d; dd += 64) s += u[i * d + dd] * v[i * d + dd];
    s = wave_sum(s);
    if (lane == 0) {
        float r = s * inv_tau;
        if (ub) r = r + ub[0] + ib[0];
        out[i] = r;
    }
}

}  // namespace loss
}  // namespace rt

using namespace rt;

namespace {
int run_loss(const void* u, const void* p, const void* q, int dtype, int64_t b, int d, int n_neg, float inv_tau,
             const float* ub, const float* ib, float we, float wb, double* loss_out, float* du, float* dp,
             float* dq, float* dub, float* dib, void* ws, size_t ws_bytes, void* stream, bool grad) {
    if (dtype != RT_F32) return RT_ERR_UNSUPPORTED;
    if (b <= 0 || d <= 0 || n_neg < 0 || !u || !p || !loss_out) return RT_ERR_INVALID;
    if (d % 8 != 0 || d > loss::kMaxD || n_neg > loss::kMaxNeg) return RT_ERR_UNSUPPORTED;
    if (n_neg > 0 && !q) return RT_ERR_INVALID;
    if (grad && (!du || !dp || (n_neg > 0 && !dq))) return RT_ERR_INVALID;
    const int n_split = static_cast<int>((b + loss::JT - 1) / loss::JT);
    const size_t need = static_cast<size_t>(n_split) * b * sizeof(float2) + static_cast<size_t>(b) * sizeof(float);
    if (!ws || ws_bytes < need) return RT_ERR_WORKSPACE;
    if ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(p)) & 15) return RT_ERR_INVALID;
    float2* part = reinterpret_cast<float2*>(ws);
    float* diag = reinterpret_cast<float*>(part + static_cast<size_t>(n_split) * b);
    const float wb_eff = n_neg > 0 ? wb : 1.f;  // in-batch alone: the loss IS the in-batch CE (weight 1)
    const float we_eff = n_neg > 0 ? we : 0.f;
    loss::Args a{static_cast<const float*>(u), static_cast<const float*>(p), static_cast<const float*>(q),
                 b, d, n_neg, inv_tau, ub, ib, we_eff, wb_eff, loss_out, du, dp, dq, dub, dib, part, diag,
                 n_split, grad};
    hipStream_t st = as_stream(stream);
    const unsigned nt = static_cast<unsigned>((b + loss::RB - 1) / loss::RB);
    hipLaunchKernelGGL(loss::loss_fwd_kernel, dim3(nt, n_split), dim3(256), 0, st, a);
    int rc = check_launch("loss_fwd_kernel");
    if (rc) return rc;
    const bool want_ib = wb_eff != 0.f;
    if (!want_ib) return RT_OK;  // contrastive_loss alone
    // forward-only calls still need launch 2's row pass for the in-batch loss value
    const dim3 grid(nt, n_split, grad ? 2 : 1);
    const int dt = (d + 31) / 32;
    switch (dt) {
        case 1: hipLaunchKernelGGL(loss::loss_bwd_kernel<1>, grid, dim3(256), 0, st, a, wb_eff, true); break;
        case 2: hipLaunchKernelGGL(loss::loss_bwd_kernel<2>, grid, dim3(256), 0, st, a, wb_eff, true); break;
        case 3:
        case 4: hipLaunchKernelGGL(loss::loss_bwd_kernel<4>, grid, dim3(256), 0, st, a, wb_eff, true); break;
        default: hipLaunchKernelGGL(loss::loss_bwd_kernel<8>, grid, dim3(256), 0, st, a, wb_eff, true); break;
    }
    return check_launch("loss_bwd_kernel");
}
}  // namespace

extern "C" size_t rt_twotower_loss_workspace_bytes(int64_t b, int d) {
    (void)d;
    if (b <= 0) return 256;
    const int64_t n_split = (b + loss::JT - 1) / loss::JT;
    return static_cast<size_t>(n_split) * b * sizeof(float2) + static_cast<size_t>(b) * sizeof(float) + 256;
}


extern "C" int rt_twotower_loss_fwd_bwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                                        int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                                        float w_explicit, float w_in_batch, double* loss_out, float* du, float* dp,
                                        float* dq, float* d_user_bias, float* d_item_bias, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    return run_loss(u, p, q, dtype, b, d, n_neg, inv_tau, user_bias, item_bias, w_explicit, w_in_batch, loss_out,
                    du, dp, dq, d_user_bias, d_item_bias, workspace, workspace_bytes, stream, true);
}

extern "C" int rt_twotower_loss_fwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                                    int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                                    float w_explicit, float w_in_batch, double* loss_out, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    return run_loss(u, p, q, dtype, b, d, n_neg, inv_tau, user_bias, item_bias, w_explicit, w_in_batch, loss_out,
                    nullptr, nullptr, nullptr, nullptr, nullptr, workspace, workspace_bytes, stream, false);
}

extern "C" int rt_similarity_f32(const float* u, const float* v, int64_t b, int d, float inv_tau,
                                 const float* user_bias, const float* item_bias, float* out, void* stream) {
    if (b < 0 || d <= 0 || !u || !v || !out) return RT_ERR_INVALID;
    if ((user_bias == nullptr) != (item_bias == nullptr)) return RT_ERR_INVALID;
    if (b == 0) return RT_OK;
    hipLaunchKernelGGL(loss::similarity_kernel, dim3(static_cast<unsigned>((b + 3) / 4)), dim3(256), 0,
                       as_stream(stream), u, v, b, d, inv_tau, user_bias, item_bias, out);
    return check_launch("similarity_kernel");
}
