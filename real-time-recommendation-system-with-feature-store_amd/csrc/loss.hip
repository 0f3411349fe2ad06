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
    for (int s = 0; s < D / 2; s += 4) {
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
    float we, wb;
    double* loss;
    float* du; float* dp; float* dq; float* dub; float* dib;
    float* lse;  // workspace [b]
    bool grad;
};

// ---------------------------------------------------------------- launch 1
__global__ __launch_bounds__(256) void loss_rows_kernel(Args a) {
    __shared__ float diag[RB];
    __shared__ float negs[4][kMaxNeg];
    __shared__ float red_m[4][RB], red_l[4][RB];
    __shared__ double red_loss[4][2];
    __shared__ float red_bias[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int64_t i0 = static_cast<int64_t>(blockIdx.x) * RB;
    const int D = a.d;
    const float bias = (a.ub ? a.ub[0] : 0.f) + (a.ib ? a.ib[0] : 0.f);
    const float inv_b = 1.f / static_cast<float>(a.b);
    double loss_e = 0.0;
    float dbias_acc = 0.f;

    // ---- explicit negatives: one wave per user, lanes over d ----
    for (int ii = w * 8; ii < w * 8 + 8; ++ii) {
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
        if (lane == 0) diag[ii] = dup;
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
        float mx = pos;
        for (int j = 0; j < a.n_neg; ++j) {
            const float* qr = a.q + (i * a.n_neg + j) * D;
            float pq = 0.f;
#pragma unroll
            for (int t = 0; t < kMaxD / 64; ++t) {
                const int dd = lane + 64 * t;
                if (dd < D) pq += uv[t] * qr[dd];
            }
            const float nv = wave_sum(pq) * a.inv_tau;
            if (lane == 0) negs[w][j] = nv;
            mx = fmaxf(mx, nv);
        }
        wave_lds_sync();
        float se = expf(pos - mx);
        for (int j = 0; j < a.n_neg; ++j) se += expf(negs[w][j] - mx);
        const float lse = mx + logf(se);
        if (lane == 0) loss_e += static_cast<double>(lse - pos);
        if (!a.grad) continue;
        const float dpos = a.we * inv_b * (expf(pos - lse) - 1.f);
        if (lane == 0) dbias_acc += dpos;
        float duv[kMaxD / 64];
#pragma unroll
        for (int t = 0; t < kMaxD / 64; ++t) duv[t] = dpos * pv[t];
        for (int j = 0; j < a.n_neg; ++j) {
            const float dn = a.we * inv_b * expf(negs[w][j] - lse);
            const float* qr = a.q + (i * a.n_neg + j) * D;
            float* dqr = a.dq + (i * a.n_neg + j) * D;
#pragma unroll
            for (int t = 0; t < kMaxD / 64; ++t) {
                const int dd = lane + 64 * t;
                if (dd < D) {
                    duv[t] += dn * qr[dd];
                    dqr[dd] = dn * uv[t] * a.inv_tau;
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
    __syncthreads();

    // ---- in-batch row log-sum-exp: S^T tiles [32 items j × 32 users i] ----
    float om = -INFINITY, ol = 0.f;
    const int64_t ntiles = (a.b + 31) / 32;
    for (int64_t t = w; t < ntiles; t += 4) {
        const f32x16 acc = dot_tile(a.p, t * 32, a.b, a.u, i0, a.b, D);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t j = t * 32 + tile_row(r, h);
            if (j < a.b) {
                const float s = acc[r] * a.inv_tau;
                if (s > om) { ol = ol * expf(om - s) + 1.f; om = s; }
                else ol += expf(s - om);
            }
        }
    }
    {   // merge the two half-waves (same user column)
        const float m2 = __shfl_xor(om, 32, 64), l2 = __shfl_xor(ol, 32, 64);
        const float mm = fmaxf(om, m2);
        ol = (mm == -INFINITY) ? 0.f : ol * expf(om - mm) + l2 * expf(m2 - mm);
        om = mm;
    }
    if (h == 0) { red_m[w][c] = om; red_l[w][c] = ol; }
    __syncthreads();
    double loss_b = 0.0;
    if (w == 0 && h == 0) {
        float mm = -INFINITY;
        for (int x = 0; x < 4; ++x) mm = fmaxf(mm, red_m[x][c]);
        float ll = 0.f;
        for (int x = 0; x < 4; ++x)
            if (red_m[x][c] != -INFINITY) ll += red_l[x][c] * expf(red_m[x][c] - mm);
        const int64_t i = i0 + c;
        if (i < a.b) {
            const float lse = mm + logf(ll);
            a.lse[i] = lse;
            loss_b = static_cast<double>(lse - diag[c]);
        }
    }
    // ---- block reduction of the losses / bias grad ----
    loss_e = wave_sum(loss_e);
    loss_b = wave_sum(loss_b);
    const float db = wave_sum(dbias_acc);
    if (lane == 0) { red_loss[w][0] = loss_e; red_loss[w][1] = loss_b; red_bias[w] = db; }
    __syncthreads();
    if (tid == 0) {
        double le = 0.0, lb = 0.0;
        float dbs = 0.f;
        for (int x = 0; x < 4; ++x) { le += red_loss[x][0]; lb += red_loss[x][1]; dbs += red_bias[x]; }
        const double inv_bd = 1.0 / static_cast<double>(a.b);
        atomicAdd(&a.loss[1], le * inv_bd);
        atomicAdd(&a.loss[2], lb * inv_bd);
        atomicAdd(&a.loss[0], (a.n_neg > 0 ? a.we * le * inv_bd : 0.0) + (a.n_neg > 0 ? a.wb : 1.f) * lb * inv_bd);
        if (a.grad && a.n_neg > 0) {
            if (a.dub) atomicAdd(a.dub, dbs);
            if (a.dib) atomicAdd(a.dib, dbs);
        }
    }
}

// ---------------------------------------------------------------- launch 2
template <int DT>  // D/32 output tiles per wave accumulator
__global__ __launch_bounds__(256) void loss_inbatch_bwd_kernel(Args a, float wb_eff) {
    __shared__ float Ds[4][32][33];
    __shared__ float red[32 * (kMaxD + 1)];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int D = a.d;
    const int64_t nb = (a.b + 31) / 32;
    const bool row_pass = blockIdx.x < nb;
    const int64_t f0 = (row_pass ? blockIdx.x : blockIdx.x - nb) * static_cast<int64_t>(RB);  // fixed 32 rows
    const float* Str = row_pass ? a.p : a.u;      // streamed operand
    const float scale = wb_eff / static_cast<float>(a.b);
    f32x16 acc[DT];
#pragma unroll
    for (int x = 0; x < DT; ++x) acc[x] = f32x16{};
    // row pass: tile element (row = item j, col = user i) → lse of the user = lane's column
    const float lse_col = (row_pass && f0 + c < a.b) ? a.lse[f0 + c] : 0.f;
    const int64_t ntiles = nb;
    for (int64_t t = w; t < ntiles; t += 4) {
        const f32x16 st = row_pass ? dot_tile(a.p, t * 32, a.b, a.u, f0, a.b, D)    // (j, i)
                                   : dot_tile(a.u, t * 32, a.b, a.p, f0, a.b, D);   // (i, j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rr = tile_row(r, h);
            const int64_t srow = t * 32 + rr;   // streamed index
            const int64_t fcol = f0 + c;        // fixed index
            float ds = 0.f;
            if (srow < a.b && fcol < a.b) {
                const float lse = row_pass ? lse_col : a.lse[srow];
                const float pr = expf(st[r] * a.inv_tau - lse);
                ds = scale * (pr - (srow == fcol ? 1.f : 0.f));
            }
            Ds[w][c][rr] = ds;  // [fixed][streamed]
        }
        wave_lds_sync();
        // acc[dt] (fixed f × d) += Σ_s Ds[f][s] · Str[t*32 + s][d]
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            const int dcol = dt * 32 + c;
            for (int s = 0; s < 16; ++s) {
                const int ks = 2 * s + h;
                const int64_t sr = t * 32 + ks;
                const float bv = (sr < a.b && dcol < D) ? Str[sr * D + dcol] : 0.f;
                acc[dt] = mfma(Ds[w][c][ks], bv, acc[dt]);
            }
        }
        wave_lds_sync();
    }
    // reduce the 4 wave partials through LDS: red[f][d]
    for (int e = tid; e < 32 * (kMaxD + 1); e += 256) red[e] = 0.f;
    __syncthreads();
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) atomicAdd(&red[tile_row(r, h) * (kMaxD + 1) + dt * 32 + c], acc[dt][r]);
    __syncthreads();
    float* out = row_pass ? a.du : a.dp;
    for (int e = tid; e < 32 * D; e += 256) {
        const int f = e / D, dd = e % D;
        const int64_t gi = f0 + f;
        if (gi < a.b) out[gi * D + dd] += red[f * (kMaxD + 1) + dd] * a.inv_tau;
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
    if (!ws || ws_bytes < static_cast<size_t>(b) * sizeof(float)) return RT_ERR_WORKSPACE;
    if ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(p)) & 15) return RT_ERR_INVALID;
    loss::Args a{static_cast<const float*>(u), static_cast<const float*>(p), static_cast<const float*>(q),
                 b, d, n_neg, inv_tau, ub, ib, we, wb, loss_out, du, dp, dq, dub, dib,
                 static_cast<float*>(ws), grad};
    hipStream_t st = as_stream(stream);
    const unsigned nb = static_cast<unsigned>((b + loss::RB - 1) / loss::RB);
    hipLaunchKernelGGL(loss::loss_rows_kernel, dim3(nb), dim3(256), 0, st, a);
    int rc = check_launch("loss_rows_kernel");
    if (rc || !grad) return rc;
    const float wb_eff = n_neg > 0 ? wb : 1.f;  // in-batch only: the loss IS the in-batch CE
    if (wb_eff == 0.f) return RT_OK;            // contrastive_loss alone
    const int dt = (d + 31) / 32;
    switch (dt) {
        case 1: hipLaunchKernelGGL(loss::loss_inbatch_bwd_kernel<1>, dim3(2 * nb), dim3(256), 0, st, a, wb_eff); break;
        case 2: hipLaunchKernelGGL(loss::loss_inbatch_bwd_kernel<2>, dim3(2 * nb), dim3(256), 0, st, a, wb_eff); break;
        case 3:
        case 4: hipLaunchKernelGGL(loss::loss_inbatch_bwd_kernel<4>, dim3(2 * nb), dim3(256), 0, st, a, wb_eff); break;
        default: hipLaunchKernelGGL(loss::loss_inbatch_bwd_kernel<8>, dim3(2 * nb), dim3(256), 0, st, a, wb_eff); break;
    }
    return check_launch("loss_inbatch_bwd_kernel");
}
}  // namespace

extern "C" size_t rt_twotower_loss_workspace_bytes(int64_t b, int d) {
    (void)d;
    return static_cast<size_t>(b > 0 ? b : 1) * sizeof(float) + 256;
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
