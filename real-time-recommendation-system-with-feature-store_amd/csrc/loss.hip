// Two-tower losses, fused forward + backward (fp32 scores and gradients as
// three-piece bf16 MFMA sextets, split3.h).
//
// Replaces (src/models/two_tower.py):
//   compute_similarity      :380-404   → rt_similarity_f32
//   contrastive_loss        :406-451   (explicit negatives, biases on the positive logit only)
//   in_batch_negative_loss  :453-479   (S = U·Pᵀ/τ, CE with diagonal labels)
// and the trainer's mixing 0.7·explicit + 0.3·in-batch
// (src/training/trainers/two_tower.py:111-137), forward AND backward.
//
// Block geometry of the in-batch part: a FIXED tile of 32 rows (users, or items
// in the column pass) whose fragments sit in registers, and a STREAMED span of
// 256 rows: each wave stages two 32-row tiles through its own LDS slice (all
// loads of a tile in flight at once, the next tile prefetched into registers
// while the current one is on the MFMAs).
// Launch 1 (B/32 × B/256 blocks): per-span partial row log-sum-exp of S = U·Pᵀ/τ
//   (online max/sum, S never stored), plus the explicit contrastive CE with its
//   gradients for a strided subset of the block's users.
// Launch 2 (2 × B/32 × B/256 blocks): S tiles are recomputed; the accumulator
//   of an S tile is directly the A operand of the next MFMA (the k order over
//   the streamed rows follows the accumulator layout), so dU = dS·P (row pass)
//   and dP = dSᵀ·U (column pass) need no LDS transpose; dS = w/B·(softmax − I).
//   The 4 waves' partials are summed through LDS, one atomic per element per span.
// Every MFMA operand is an fp32 value taken as its three bf16 pieces; the
// k-order of an S chain is that of the 32x32x16 MFMA (lane half h holds
// k = 16kb + 8h .. +7 of k-block kb), so every fragment is two contiguous float4.
#include <float.h>

#include "rt_common.h"
#include "split3.h"

namespace rt {
size_t ib16_workspace_bytes(int64_t b, int64_t nx, int d);
int ib16_run(const void* u, const void* p, int dtype, int64_t b, int64_t nx, int d, int64_t off, float inv_tau,
             double* loss_out, float* du, float* dp, void* ws, size_t ws_bytes, hipStream_t st);
namespace loss {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int RB = 32;        // users (or items) per block
constexpr int kMaxD = 256;
constexpr int kMaxNeg = 64;
constexpr int NG = 16;  // negatives reduced together


__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct Args {
    const void* u; const void* p; const void* q;  // element type = the kernel's T
    int64_t b; int d; int n_neg; float inv_tau;
    const float* ub; const float* ib;
    float we, wb;       // weights of the explicit / in-batch terms in loss_out[0]
    double* loss;
    float* du; float* dp; float* dq; float* dub; float* dib;
    float2* part;       // workspace [n_split][b]: per-split (max, sum exp) of S rows
    float* diag;        // workspace [b]: S_ii = u_i·p_i / tau
    float* expl;        // workspace [b]: explicit CE term lse_i − pos_i
    float* dposv;       // workspace [b]: d loss / d pos_i (= d loss / d bias share of user i)
    int64_t nx;         // rows of p (in-batch items); == b for the square reference loss
    int64_t off;        // label of user i is item off + i (DP shard of a global batch)
    int n_split;        // streamed spans of SPAN rows (items)
    int ib_blocks;      // launch-1 in-batch block rows (n_split, or 0 without the in-batch term)
    bool grad;
};

constexpr int SPAN = 256;  // streamed rows per block (4 waves x 2 tiles of 32)
constexpr int LDP = 4;     // LDS row pad (floats): conflict-free ds_read_b128 of 16 rows

// ---- in-batch building blocks (DP = D padded to a multiple of 32) ----------
// one wave loads 32 rows x DP floats of M (rows >= n and cols >= D read as 0)
// 4 consecutive elements widened to fp32 (16-bit types: one 8-byte load)
template <typename T>
__device__ __forceinline__ float4 load4(const T* __restrict__ p) {
    if constexpr (sizeof(T) == 4) {
        return *reinterpret_cast<const float4*>(p);
    } else {
        const uint2 r = *reinterpret_cast<const uint2*>(p);
        const T* e = reinterpret_cast<const T*>(&r);
        return make_float4(to_f32(e[0]), to_f32(e[1]), to_f32(e[2]), to_f32(e[3]));
    }
}

template <int DP, typename T>
__device__ __forceinline__ void load_rows(const T* __restrict__ M, int64_t r0, int64_t n, int D,
                                          float4 (&v)[DP / 8]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < DP / 8; ++u) {
        const int e = lane + 64 * u;
        const int row = e / (DP / 4), c = (e % (DP / 4)) * 4;
        const int64_t gr = r0 + row;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < n && c < D) v[u] = load4<T>(M + gr * D + c);
    }
}
template <int DP>
__device__ __forceinline__ void store_rows(float* __restrict__ S, const float4 (&v)[DP / 8]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < DP / 8; ++u) {
        const int e = lane + 64 * u;
        const int row = e / (DP / 4), c = (e % (DP / 4)) * 4;
        *reinterpret_cast<float4*>(S + row * (DP + LDP) + c) = v[u];
    }
}
// fixed-row pieces per 16-deep k-block (fp32 products on the bf16 MFMA,
// split3.h): lane (c, h) holds the split of F[f0 + c][16kb + 8h .. 16kb + 8h + 7]
using fsplit::Pieces;
using fsplit::split8;
using fsplit::mfma3;
template <int DP, typename T>
__device__ __forceinline__ void load_fixed3(const T* __restrict__ F, int64_t f0, int64_t n, int D,
                                            Pieces (&pf)[DP / 16]) {
    const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const int64_t r = f0 + c;
#pragma unroll
    for (int kb = 0; kb < DP / 16; ++kb) {
        const int k = 16 * kb + 8 * h;  // D % 8 == 0: a k-block half is all in or all out
        float4 u = make_float4(0.f, 0.f, 0.f, 0.f), v = u;
        if (r < n && k < D) {
            u = load4<T>(F + r * D + k);
            v = load4<T>(F + r * D + k + 4);
        }
        const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        pf[kb] = split8(x);
    }
}
// acc[r] = <streamed row tile_row(r,h) of Ss, fixed row (lane & 31)> (raw dots),
// one bf16 MFMA sextet per 16-deep k-block
template <int DP>
__device__ __forceinline__ f32x16 s_tile3(const float* __restrict__ Ss, const Pieces (&pf)[DP / 16]) {
    const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const float* ap = Ss + c * (DP + LDP) + 8 * h;
    f32x16 acc = {};
#pragma unroll
    for (int kb = 0; kb < DP / 16; ++kb) {
        const float4 u = *reinterpret_cast<const float4*>(ap + 16 * kb);
        const float4 v = *reinterpret_cast<const float4*>(ap + 16 * kb + 4);
        const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        acc = mfma3(split8(x), pf[kb], acc);
    }
    return acc;
}
// dynamic LDS of the in-batch kernels: 4 waves x 32 rows x (DP + LDP) floats
template <int DP>
constexpr size_t inb_lds_bytes() { return static_cast<size_t>(4) * 32 * (DP + LDP) * sizeof(float); }

// ---------------------------------------------------------------- launch 1
// block (it, js < n_split): in-batch partial row log-sum-exp of users
// [32it, 32it+32) over items [256js, 256js+256);
// block (it, n_split + e), e < 8: explicit contrastive CE (+ gradients) of users
// 32it + 4e + w, one wave per user, the negative rows loaded once.
template <int DP, typename T>
__global__ __launch_bounds__(256) void loss_fwd_kernel(Args a) {
    const T* __restrict__ U = static_cast<const T*>(a.u);
    const T* __restrict__ P = static_cast<const T*>(a.p);
    const T* __restrict__ Qn = static_cast<const T*>(a.q);
    extern __shared__ __attribute__((aligned(16))) float sm_f[];
    __shared__ float negs[4][kMaxNeg];
    __shared__ float red_m[4][RB], red_l[4][RB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int it = blockIdx.x, js = blockIdx.y;
    const int64_t i0 = static_cast<int64_t>(it) * RB;
    const int D = a.d;
    const float bias = (a.ub ? a.ub[0] : 0.f) + (a.ib ? a.ib[0] : 0.f);
    const float inv_b = 1.f / static_cast<float>(a.b);

    if (js < a.ib_blocks) {
        // ---- in-batch partial lse: S^T tiles (items j × users i) ----
        float* Ss = sm_f + w * 32 * (DP + LDP);
        Pieces pf[DP / 16];
        load_fixed3<DP, T>(U, i0, a.b, D, pf);
        const int64_t t0 = static_cast<int64_t>(js) * SPAN + 32 * w, t1 = t0 + 128;
        float4 buf[DP / 8];
        load_rows<DP, T>(P, t0, a.nx, D, buf);
        float om = -INFINITY, ol = 0.f;
#pragma unroll 1
        for (int q = 0; q < 2; ++q) {
            const int64_t tt = q == 0 ? t0 : t1;
            if (tt >= a.nx) break;  // wave-uniform
            store_rows<DP>(Ss, buf);
            wave_lds_sync();
            if (q == 0 && t1 < a.nx) load_rows<DP, T>(P, t1, a.nx, D, buf);  // prefetch
            const f32x16 acc = s_tile3<DP>(Ss, pf);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (tt + tile_row(r, h) < a.nx) {
                    const float sv = acc[r] * a.inv_tau;
                    if (sv > om) { ol = ol * expf(om - sv) + 1.f; om = sv; }
                    else ol += expf(sv - om);
                }
            }
            wave_lds_sync();
        }
        const float m2 = __shfl_xor(om, 32, 64), l2 = __shfl_xor(ol, 32, 64);
        const float mm = fmaxf(om, m2);
        ol = (mm == -INFINITY) ? 0.f : ol * expf(om - mm) + l2 * expf(m2 - mm);
        if (h == 0) { red_m[w][c] = mm; red_l[w][c] = ol; }
        __syncthreads();
        if (w == 0 && h == 0 && i0 + c < a.b) {
            float m3 = -INFINITY;
            for (int x = 0; x < 4; ++x) m3 = fmaxf(m3, red_m[x][c]);
            float ll = 0.f;
            if (m3 != -INFINITY)
                for (int x = 0; x < 4; ++x) ll += red_l[x][c] * expf(red_m[x][c] - m3);
            a.part[static_cast<int64_t>(js) * a.b + i0 + c] = make_float2(m3, ll);
        }
        return;
    }

    // ---- explicit negatives: blocks js >= n_split, one user per wave ----
    const int64_t i = i0 + 4 * (js - a.ib_blocks) + w;
    if (i >= a.b) return;
    const T* ur = U + i * D;
    const T* pr = P + (a.off + i) * D;  // the user's positive (its label)
    constexpr int V = kMaxD / 64;
    float uv[V], pv[V];
    float part = 0.f;
#pragma unroll
    for (int t = 0; t < V; ++t) {
        const int dd = lane + 64 * t;
        uv[t] = dd < D ? to_f32(ur[dd]) : 0.f;
        pv[t] = dd < D ? to_f32(pr[dd]) : 0.f;
        part += uv[t] * pv[t];
    }
    // the first NG negative rows stay in registers for the gradient pass
    float qv[NG][V];
    auto load_q = [&](int g0) {
#pragma unroll
        for (int jj = 0; jj < NG; ++jj) {
            const int j = g0 + jj;
            const T* qr = Qn + (i * a.n_neg + (j < a.n_neg ? j : 0)) * D;
#pragma unroll
            for (int t = 0; t < V; ++t) {
                const int dd = lane + 64 * t;
                qv[jj][t] = (j < a.n_neg && dd < D) ? to_f32(qr[dd]) : 0.f;
            }
        }
    };
    if (a.n_neg > 0) load_q(0);  // in flight with the positive dot's reduction
    const float dup = wave_sum(part) * a.inv_tau;
    if (lane == 0) a.diag[i] = dup;
    if (a.n_neg <= 0) {
        if (a.grad) {
#pragma unroll
            for (int t = 0; t < V; ++t) {
                const int dd = lane + 64 * t;
                if (dd < D) { a.du[i * D + dd] = 0.f; a.dp[i * D + dd] = 0.f; }
            }
        }
        return;
    }
    const float pos = dup + bias;
    float mx = pos;
    for (int g0 = 0; g0 < a.n_neg; g0 += NG) {
        if (g0 > 0) load_q(g0);
        float part_j[NG];
#pragma unroll
        for (int jj = 0; jj < NG; ++jj) {
            part_j[jj] = 0.f;
#pragma unroll
            for (int t = 0; t < V; ++t) part_j[jj] += uv[t] * qv[jj][t];
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
    // per-user terms; launch 2 reduces them (one atomic per 32 users)
    const float dpos = a.we * inv_b * (expf(pos - lse) - 1.f);
    if (lane == 0) {
        a.expl[i] = lse - pos;
        a.dposv[i] = dpos;
    }
    if (!a.grad) return;
    float duv[V];
#pragma unroll
    for (int t = 0; t < V; ++t) duv[t] = dpos * pv[t];
    for (int g0 = 0; g0 < a.n_neg; g0 += NG) {
        if (a.n_neg > NG) load_q(g0);  // registers still hold group 0 when n_neg <= NG
#pragma unroll
        for (int jj = 0; jj < NG; ++jj) {
            const int j = g0 + jj;
            if (j >= a.n_neg) break;
            const float dn = a.we * inv_b * expf(negs[w][j] - lse);
            float* dqr = a.dq + (i * a.n_neg + j) * D;
#pragma unroll
            for (int t = 0; t < V; ++t) {
                const int dd = lane + 64 * t;
                if (dd < D) {
                    duv[t] += dn * qv[jj][t];
                    dqr[dd] = dn * uv[t] * a.inv_tau;
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < V; ++t) {
        const int dd = lane + 64 * t;
        if (dd < D) {
            a.du[i * D + dd] = duv[t] * a.inv_tau;
            a.dp[i * D + dd] = dpos * uv[t] * a.inv_tau;
        }
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
// blockIdx.z = 0: row pass, fixed 32 users, dU += dS · P over the span's items
// blockIdx.z = 1: column pass, fixed 32 items, dP += dSᵀ · U over the span's users
// (dS = wb/B·(softmax(S) − I)); one atomic add per output element per span.
template <int DP, typename T>
__global__ __launch_bounds__(256) void loss_bwd_kernel(Args a, float wb_eff, bool add_loss) {
    constexpr int DT = DP / 32;
    extern __shared__ __attribute__((aligned(16))) float sm_b[];
    __shared__ float lse_s[SPAN];  // column pass: the span's streamed users
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int D = a.d;
    const bool row_pass = blockIdx.z == 0;
    const int64_t f0 = static_cast<int64_t>(blockIdx.x) * RB;    // fixed tile
    const int64_t s0 = static_cast<int64_t>(blockIdx.y) * SPAN;  // streamed span
    // row pass: fixed users (b), streamed items (nx); column pass: the reverse
    const int64_t n_fixed = row_pass ? a.b : a.nx, n_str = row_pass ? a.nx : a.b;
    if (f0 >= n_fixed || s0 >= n_str) {  // grid covers the larger of the two passes
        if (!(row_pass && blockIdx.y == 0 && f0 < a.b)) return;
    }
    const T* Fm = static_cast<const T*>(row_pass ? a.u : a.p);
    const T* Sm = static_cast<const T*>(row_pass ? a.p : a.u);
    const float scale = wb_eff / static_cast<float>(a.b);
    float lse_fixed = 0.f;  // row pass: lse of user f0 + c
    const bool ib = wb_eff != 0.f;
    if (row_pass) {
        const int64_t i = f0 + c;
        if (ib && i < a.b) lse_fixed = combine_lse(a.part, a.n_split, a.b, i);
        if (add_loss && blockIdx.y == 0 && w == 0) {
            // the loss scalars and bias grads of these 32 users: one atomic each
            double li = 0.0, le = 0.0;
            float dpb = 0.f;
            if (h == 0 && i < a.b) {
                if (ib) li = static_cast<double>(lse_fixed - a.diag[i]) / static_cast<double>(a.b);
                if (a.n_neg > 0) {
                    le = static_cast<double>(a.expl[i]) / static_cast<double>(a.b);
                    dpb = a.dposv[i];
                }
            }
            li = wave_sum(li);
            le = wave_sum(le);
            dpb = wave_sum(dpb);
            if (lane == 0) {
                if (ib) atomicAdd(&a.loss[2], li);
                if (a.n_neg > 0) atomicAdd(&a.loss[1], le);
                atomicAdd(&a.loss[0], static_cast<double>(wb_eff) * li + static_cast<double>(a.we) * le);
                if (a.grad && a.n_neg > 0) {
                    if (a.dub) atomicAdd(a.dub, dpb);
                    if (a.dib) atomicAdd(a.dib, dpb);
                }
            }
        }
    } else {
        const int64_t i = s0 + tid;
        lse_s[tid] = i < a.b ? combine_lse(a.part, a.n_split, a.b, i) : 0.f;  // streamed users
    }
    __syncthreads();
    if (!a.grad || !ib || f0 >= n_fixed || s0 >= n_str) return;

    float* Ss = sm_b + w * 32 * (DP + LDP);
    Pieces pf[DP / 16];
    load_fixed3<DP, T>(Fm, f0, n_fixed, D, pf);
    const int64_t t0 = s0 + 32 * w, t1 = t0 + 128;
    float4 buf[DP / 8];
    load_rows<DP, T>(Sm, t0, n_str, D, buf);
    f32x16 acc[DT];
#pragma unroll
    for (int x = 0; x < DT; ++x) acc[x] = f32x16{};
#pragma unroll 1
    for (int q = 0; q < 2; ++q) {
        const int64_t tt = q == 0 ? t0 : t1;
        if (tt >= n_str) break;  // wave-uniform
        store_rows<DP>(Ss, buf);
        wave_lds_sync();
        if (q == 0 && t1 < n_str) load_rows<DP, T>(Sm, t1, n_str, D, buf);  // prefetch
        // st[r]: streamed row tile_row(r,h) x fixed col c
        const f32x16 st = s_tile3<DP>(Ss, pf);
        float ds[16];
        const int64_t fcol = f0 + c;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rr = tile_row(r, h);
            const int64_t srow = tt + rr;
            float v = 0.f;
            if (srow < n_str && fcol < n_fixed) {
                const float lse = row_pass ? lse_fixed : lse_s[32 * w + 128 * q + rr];
                // label: item off + user  (row pass: srow item, fcol user; column pass: the reverse)
                const bool label = row_pass ? (srow == a.off + fcol) : (fcol == a.off + srow);
                v = scale * (expf(st[r] * a.inv_tau - lse) - (label ? 1.f : 0.f));
            }
            ds[r] = v;
        }
        // dF[fixed c][d] += Σ_r dS[fixed c][streamed tile_row(r,h)] · Str[tile_row(r,h)][d]:
        // k-block b of the sextets = accumulator registers 8b..8b+7 of both lane
        // halves (streamed rows 16b..16b+15), so dS enters as it lies (lane-local)
        Pieces pds[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const float x[8] = {ds[8 * b], ds[8 * b + 1], ds[8 * b + 2], ds[8 * b + 3],
                                ds[8 * b + 4], ds[8 * b + 5], ds[8 * b + 6], ds[8 * b + 7]};
            pds[b] = split8(x);
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float y[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) y[j] = Ss[tile_row(8 * b + j, h) * (DP + LDP) + dt * 32 + c];
                acc[dt] = mfma3(pds[b], split8(y), acc[dt]);
            }
        }
        wave_lds_sync();
    }
    // ---- sum the 4 waves' [32 fixed x DP] partials through LDS, one atomic each ----
    __syncthreads();  // every wave done with its Ss slice
    float* red = sm_b;  // [4][DT*16][64]
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(w * DT * 16 + dt * 16 + r) * 64 + lane] = acc[dt][r];
    __syncthreads();
    float* out = row_pass ? a.du : a.dp;
    for (int p = tid; p < DT * 16 * 64; p += 256) {
        const int v = p >> 6, l = p & 63;
        const float t = red[v * 64 + l] + red[(DT * 16 + v) * 64 + l] + red[(2 * DT * 16 + v) * 64 + l] +
                        red[(3 * DT * 16 + v) * 64 + l];
        const int dt = v >> 4, r = v & 15;
        const int64_t gi = f0 + tile_row(r, l >> 5);
        const int dd = dt * 32 + (l & 31);
        if (gi < n_fixed && dd < D) atomicAdd(&out[gi * D + dd], t * a.inv_tau);
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
// allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); set once per kernel
template <typename K>
void allow_lds(K kernel, size_t bytes) {
    static size_t set = 0;
    if (bytes > set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(bytes));
        set = bytes;
    }
}

template <int DP, typename T>
int launch_loss(const loss::Args& a, dim3 grid1, dim3 grid2, float wb_eff, hipStream_t st) {
    const size_t lds = loss::inb_lds_bytes<DP>();
    allow_lds(loss::loss_fwd_kernel<DP, T>, lds);
    hipLaunchKernelGGL((loss::loss_fwd_kernel<DP, T>), grid1, dim3(256), lds, st, a);
    const int rc = check_launch("loss_fwd_kernel");
    if (rc) return rc;
    allow_lds(loss::loss_bwd_kernel<DP, T>, lds);
    hipLaunchKernelGGL((loss::loss_bwd_kernel<DP, T>), grid2, dim3(256), lds, st, a, wb_eff, true);
    return check_launch("loss_bwd_kernel");
}

template <typename T>
int launch_loss_d(const loss::Args& a, int dp32, dim3 grid1, dim3 grid2, float wb_eff, hipStream_t st) {
    switch (dp32) {
        case 32: return launch_loss<32, T>(a, grid1, grid2, wb_eff, st);
        case 64: return launch_loss<64, T>(a, grid1, grid2, wb_eff, st);
        case 96:
        case 128: return launch_loss<128, T>(a, grid1, grid2, wb_eff, st);
        default: return launch_loss<256, T>(a, grid1, grid2, wb_eff, st);
    }
}

size_t loss_ws_bytes(int64_t b, int64_t nx) {
    const int64_t n_split = (nx + loss::SPAN - 1) / loss::SPAN;
    return static_cast<size_t>(n_split) * b * sizeof(float2) + 3 * static_cast<size_t>(b) * sizeof(float);
}

// b users; nx in-batch items (rows of p), label of user i = item off + i
int run_loss(const void* u, const void* p, const void* q, int dtype, int64_t b, int64_t nx, int64_t off, int d,
             int n_neg, float inv_tau, const float* ub, const float* ib, float we, float wb, double* loss_out,
             float* du, float* dp, float* dq, float* dub, float* dib, void* ws, size_t ws_bytes, void* stream,
             bool grad) {
    if (dtype != RT_F32 && dtype != RT_F16 && dtype != RT_BF16) return RT_ERR_INVALID;
    if (b <= 0 || d <= 0 || n_neg < 0 || !u || !p || !loss_out) return RT_ERR_INVALID;
    if (nx < b || off < 0 || off + b > nx) return RT_ERR_INVALID;
    if (d % 8 != 0 || d > loss::kMaxD || n_neg > loss::kMaxNeg) return RT_ERR_UNSUPPORTED;
    if (n_neg > 0 && !q) return RT_ERR_INVALID;
    if (grad && (!du || !dp || (n_neg > 0 && !dq))) return RT_ERR_INVALID;
    const int n_split = static_cast<int>((nx + loss::SPAN - 1) / loss::SPAN);
    if (!ws || ws_bytes < loss_ws_bytes(b, nx)) return RT_ERR_WORKSPACE;
    if ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(p)) & 15) return RT_ERR_INVALID;
    float2* part = reinterpret_cast<float2*>(ws);
    float* diag = reinterpret_cast<float*>(part + static_cast<size_t>(n_split) * b);
    const float wb_eff = n_neg > 0 ? wb : 1.f;  // in-batch alone: the loss IS the in-batch CE (weight 1)
    const float we_eff = n_neg > 0 ? we : 0.f;
    const bool want_ib = wb_eff != 0.f;
    loss::Args a{u, p, q, b, d, n_neg, inv_tau, ub, ib, we_eff, wb_eff, loss_out, du, dp, dq, dub, dib, part, diag,
                 diag + b, diag + 2 * b, nx, off, n_split, want_ib ? n_split : 0, grad};
    hipStream_t st = as_stream(stream);
    if (grad && nx != b) {  // dp rows beyond the local users get only column-pass adds
        if (hipMemsetAsync(dp, 0, static_cast<size_t>(nx) * d * sizeof(float), st) != hipSuccess)
            return check_launch("hipMemsetAsync(dp)");
    }
    const int64_t big = nx > b ? nx : b;
    const int dp32 = (d + 31) / 32 * 32;
    // launch 2 always runs: its row pass reduces the loss scalars and bias grads;
    // its grid covers both passes (fixed tiles of max(b, nx), spans of max(nx, b))
    const unsigned y2 = static_cast<unsigned>((big + loss::SPAN - 1) / loss::SPAN);
    const dim3 grid1(static_cast<unsigned>((b + loss::RB - 1) / loss::RB), a.ib_blocks + 8);
    const dim3 grid2(static_cast<unsigned>((big + loss::RB - 1) / loss::RB), want_ib ? y2 : 1,
                     (grad && want_ib) ? 2 : 1);
    switch (dtype) {
        case RT_F32: return launch_loss_d<float>(a, dp32, grid1, grid2, wb_eff, st);
        case RT_F16: return launch_loss_d<__half>(a, dp32, grid1, grid2, wb_eff, st);
        default: return launch_loss_d<__hip_bfloat16>(a, dp32, grid1, grid2, wb_eff, st);
    }
}
}  // namespace

extern "C" size_t rt_twotower_loss_workspace_bytes(int64_t b, int d) {
    (void)d;
    if (b <= 0) return 256;
    return loss_ws_bytes(b, b) + 256;
}

extern "C" size_t rt_inbatch_loss_workspace_bytes(int64_t b, int64_t n_items, int d) {
    if (b <= 0 || n_items < b || d <= 0) return 256;
    // the dtype is not part of the query: room for the fp32 path and the 16-bit MFMA path
    const size_t f32 = loss_ws_bytes(b, n_items), h16 = ib16_workspace_bytes(b, n_items, d);
    return (f32 > h16 ? f32 : h16) + 256;
}

extern "C" int rt_inbatch_loss_fwd_bwd(const void* u, const void* p, int dtype, int64_t b, int64_t n_items, int d,
                                       int64_t label_offset, float inv_tau, double* loss_out, float* du, float* dp,
                                       void* workspace, size_t workspace_bytes, void* stream) {
    if (dtype == RT_F16 || dtype == RT_BF16) {  // scores and gradients on the 16-bit MFMA (inbatch16.hip)
        if (b <= 0 || d <= 0 || !u || !p || !loss_out) return RT_ERR_INVALID;
        if (n_items < b || label_offset < 0 || label_offset + b > n_items) return RT_ERR_INVALID;
        if (d % 8 != 0 || d > loss::kMaxD) return RT_ERR_UNSUPPORTED;
        if ((du == nullptr) != (dp == nullptr)) return RT_ERR_INVALID;
        if ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(p)) & 15) return RT_ERR_INVALID;
        return ib16_run(u, p, dtype, b, n_items, d, label_offset, inv_tau, loss_out, du, dp, workspace,
                        workspace_bytes, as_stream(stream));
    }
    return run_loss(u, p, nullptr, dtype, b, n_items, label_offset, d, 0, inv_tau, nullptr, nullptr, 0.f, 1.f,
                    loss_out, du, dp, nullptr, nullptr, nullptr, workspace, workspace_bytes, stream, du != nullptr);
}


extern "C" int rt_twotower_loss_fwd_bwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                                        int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                                        float w_explicit, float w_in_batch, double* loss_out, float* du, float* dp,
                                        float* dq, float* d_user_bias, float* d_item_bias, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    return run_loss(u, p, q, dtype, b, b, 0, d, n_neg, inv_tau, user_bias, item_bias, w_explicit, w_in_batch,
                    loss_out, du, dp, dq, d_user_bias, d_item_bias, workspace, workspace_bytes, stream, true);
}

extern "C" int rt_twotower_loss_fwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                                    int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                                    float w_explicit, float w_in_batch, double* loss_out, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    return run_loss(u, p, q, dtype, b, b, 0, d, n_neg, inv_tau, user_bias, item_bias, w_explicit, w_in_batch,
                    loss_out, nullptr, nullptr, nullptr, nullptr, nullptr, workspace, workspace_bytes, stream, false);
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
