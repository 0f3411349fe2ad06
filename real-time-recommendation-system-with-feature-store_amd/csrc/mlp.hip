// Tower MLP kernels (fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32).
//
// Replaces the ATen CPU op chain of UserTower/ItemTower.forward
// (src/models/two_tower.py:56-72, 98-134, 196-212, 238-281):
//   addmm → act → batch_norm → dropout  (per hidden block), addmm, F.normalize
// and its autograd backward. Each Linear is ONE forward launch:
//   prologue  : row gather (layer 1) or the previous block's act → BatchNorm
//               (batch stats finalised from fp64 column sums) → dropout,
//               applied while staging A into LDS;
//   MFMA core : 64-row tile × full output width, K streamed in 32-wide chunks;
//   epilogue  : bias, pre-activation store, fp64 column stats of act(z) for the
//               next BatchNorm, or (final layer) the row L2 normalisation.
// Backward is two launches per Linear: (1) dz (normalize/BN/act backward) +
// dgamma/dbeta + dA = dz·W with the previous block's dropout/BN-stat epilogue,
// (2) dW = dzᵀ·A and dbias over M split across blocks, A recomputed by the
// same prologue. BN column sums go to RT_STAT_SLOTS fp64 slots (include/rtrec_hip.h).
#include "rt_common.h"

namespace rt {
namespace mlp {

typedef float f32x16 __attribute__((ext_vector_type(16)));



constexpr float kNormEps = 1e-12f;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// previous-block transform applied to every A element (forward AND backward
// recompute use this one function, so the recomputed A is bit-identical)
struct Pro {
    int mode;          // 0 raw, 1/2 act+BN(+drop), 3 act(+drop)
    int act;
    float drop_p, drop_scale;
    uint64_t seed;
    const float* scale;  // LDS [k] (modes 1/2)
    const float* shift;
};

__device__ __forceinline__ float pro_apply(const Pro& p, int64_t r, int c, float v) {
    if (p.mode == 0) return v;
    v = act_fwd(p.act, v);
    if (p.mode != 3) v = __builtin_fmaf(v, p.scale[c], p.shift[c]);
    if (p.drop_p > 0.f) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
    return v;
}

// (Σ slot[c], Σ slot[w + c]) over the RT_STAT_SLOTS fp64 slots of stride 2w, in
// slot order: all 2·RT_STAT_SLOTS loads are issued before the first add (one
// memory round trip instead of a dependent chain — the slots are written by
// memory-side atomics, so every load is an HBM/MALL latency)
__device__ __forceinline__ void slot_sums(const double* __restrict__ base, int w, int c, double& s1, double& s2) {
    double v1[RT_STAT_SLOTS], v2[RT_STAT_SLOTS];
#pragma unroll
    for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
        v1[sl] = base[static_cast<int64_t>(sl) * 2 * w + c];
        v2[sl] = base[static_cast<int64_t>(sl) * 2 * w + w + c];
    }
    s1 = 0.0;
    s2 = 0.0;
#pragma unroll
    for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
        s1 += v1[sl];
        s2 += v2[sl];
    }
}

__device__ __forceinline__ void bn_affine(float gamma, float beta, float mean, float invstd, float& scale,
                                          float& shift) {
    scale = gamma * invstd;
    shift = __builtin_fmaf(-mean, scale, beta);
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Block = 32 rows x all n columns; the transformed A tile (32 x k) lives in LDS
// for the whole reduction (A fragments by ds_read_b128), W fragments stream
// straight from L2 (float4 per lane per 4 MFMAs). The reduction index is
// permuted (lane half h covers k in [h*kh, h*kh+kh)) so each lane's operands
// are contiguous; 4 waves split the output columns.
constexpr int FM = 32;  // rows per block

__host__ __device__ __forceinline__ int pad8(int k) { return (k + 31) / 32 * 32; }  // kh % 16 == 0

template <int TPW, bool KVEC>  // 32-col tiles per wave (n <= 128*TPW); KVEC: k % 4 == 0
__global__ __launch_bounds__(256) void linear_fwd_kernel(rt_linear_fwd_args a) {
    constexpr int NT = 4 * TPW;  // column tiles in the block
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int k = a.k, n = a.n;
    const int kp = pad8(k), kh = kp / 2, lda = kp + 4;
    float* scale = sm;                   // [kp]
    float* shift = scale + kp;           // [kp]
    float* As = shift + kp;              // [FM][lda]
    float* rowpart = As + FM * lda;      // [NT][FM]
    int64_t* srow = reinterpret_cast<int64_t*>(rowpart + NT * FM);  // [FM]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * FM;
    const int64_t m = a.m;

    // BatchNorm of the previous block: this block's batch is its row segment;
    // block 0 derives every segment (it owns the save/running-stat writes,
    // applied in segment order like two sequential tower calls)
    const bool two = a.seg_split > 0;
    const int my_seg = (two && row0 >= a.seg_split) ? 1 : 0;
    if (a.prev_mode == 1 || a.prev_mode == 2) {
        const int nseg = two ? 2 : 1;
        for (int c = tid; c < k; c += 256) {
            for (int sg = 0; sg < nseg; ++sg) {
                if (blockIdx.x != 0 && sg != my_seg) continue;
                const int64_t ms = two ? (sg == 0 ? a.seg_split : m - a.seg_split) : m;
                float mean, invstd, var_f = 0.f;
                if (a.prev_mode == 1) {
                    const double* ps = a.prev_stats + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * k;
                    double s1, s2;  // slot sums in slot order
                    slot_sums(ps, k, c, s1, s2);
                    const double md = s1 / static_cast<double>(ms);
                    double vd = s2 / static_cast<double>(ms) - md * md;
                    vd = vd > 0.0 ? vd : 0.0;
                    mean = static_cast<float>(md);
                    invstd = static_cast<float>(1.0 / sqrt(vd + static_cast<double>(a.bn_eps)));
                    var_f = static_cast<float>(ms > 1 ? vd * static_cast<double>(ms) / static_cast<double>(ms - 1) : vd);
                } else {
                    mean = a.running_mean[c];
                    invstd = static_cast<float>(1.0 / sqrt(static_cast<double>(a.running_var[c]) + a.bn_eps));
                }
                if (sg == my_seg) bn_affine(a.bn_gamma[c], a.bn_beta[c], mean, invstd, scale[c], shift[c]);
                if (blockIdx.x == 0) {
                    if (c == 0 && a.prev_mode == 1 && a.num_batches_tracked) *a.num_batches_tracked += 1;
                    if (a.save_mean) a.save_mean[sg * k + c] = mean;
                    if (a.save_invstd) a.save_invstd[sg * k + c] = invstd;
                    if (a.prev_mode == 1 && a.running_mean) {
                        const float mo = a.bn_momentum;
                        a.running_mean[c] = (1.f - mo) * a.running_mean[c] + mo * mean;
                        a.running_var[c] = (1.f - mo) * a.running_var[c] + mo * var_f;
                    }
                }
            }
        }
    }
    if (tid < FM) {
        const int64_t gr = row0 + tid;
        int64_t sr = -1;
        if (gr < m) {
            sr = a.ids ? a.ids[gr] : gr;
            if (sr < 0 || sr >= a.src_rows) sr = -1;
        }
        srow[tid] = sr;
    }
    __syncthreads();
    const uint64_t seed = a.drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.drop_p, a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f, seed,
                  scale, shift};
    {   // stage the transformed A tile: float4 loads, 4 in flight per thread
        const int vpr = kp / 4;
        const int total = FM * vpr;
        const bool vec = (a.ld_src % 4) == 0 && (reinterpret_cast<uintptr_t>(a.src) & 15) == 0;
        for (int base = tid; base < total; base += 256 * 4) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const int64_t sr = srow[r];
                    if (sr >= 0 && c < k) {
                        const float* sp = a.src + sr * a.ld_src + c;
                        if (vec && c + 4 <= k) v[u] = *reinterpret_cast<const float4*>(sp);
                        else {
                            v[u].x = sp[0];
                            if (c + 1 < k) v[u].y = sp[1];
                            if (c + 2 < k) v[u].z = sp[2];
                            if (c + 3 < k) v[u].w = sp[3];
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const bool ok = srow[r] >= 0;
                    const int64_t gr = row0 + r;
                    float4 o;
                    o.x = (ok && c < k) ? pro_apply(pro, gr, c, v[u].x) : 0.f;
                    o.y = (ok && c + 1 < k) ? pro_apply(pro, gr, c + 1, v[u].y) : 0.f;
                    o.z = (ok && c + 2 < k) ? pro_apply(pro, gr, c + 2, v[u].z) : 0.f;
                    o.w = (ok && c + 3 < k) ? pro_apply(pro, gr, c + 3, v[u].w) : 0.f;
                    *reinterpret_cast<float4*>(As + r * lda + c) = o;
                }
            }
        }
    }
    __syncthreads();

    f32x16 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x16{};
    const float* ap = As + c32 * lda + h * kh;
    const float* wrow[TPW];
    bool tile_on[TPW], row_ok[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        tile_on[i] = (w + 4 * i) * 32 < n;  // wave-uniform
        const int nn = (w + 4 * i) * 32 + c32;
        row_ok[i] = nn < n;
        wrow[i] = a.w + static_cast<int64_t>(row_ok[i] ? nn : 0) * k;
    }
    // 16 k-steps per iteration (kh % 16 == 0); the W fragments of the next
    // iteration are loaded during this one's MFMAs (register double buffer)
    float4 wv[TPW][4], wn[TPW][4];
    auto load_w = [&](int s, float4 (&dst)[TPW][4]) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kk = h * kh + s + 4 * j;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (tile_on[i] && row_ok[i]) {
                    const float* wr = wrow[i] + kk;
                    if constexpr (KVEC) {
                        if (kk < k) v = *reinterpret_cast<const float4*>(wr);
                    } else {
                        if (kk < k) v.x = wr[0];
                        if (kk + 1 < k) v.y = wr[1];
                        if (kk + 2 < k) v.z = wr[2];
                        if (kk + 3 < k) v.w = wr[3];
                    }
                }
                dst[i][j] = v;
            }
    };
    load_w(0, wn);
    for (int s = 0; s < kh; s += 16) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) wv[i][j] = wn[i][j];
        if (s + 16 < kh) load_w(s + 16, wn);
        float4 av[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) av[j] = *reinterpret_cast<const float4*>(ap + s + 4 * j);
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            if (!tile_on[i]) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i] = mfma(av[j].x, wv[i][j].x, acc[i]);
                acc[i] = mfma(av[j].y, wv[i][j].y, acc[i]);
                acc[i] = mfma(av[j].z, wv[i][j].z, acc[i]);
                acc[i] = mfma(av[j].w, wv[i][j].w, acc[i]);
            }
        }
    }

    // ---- epilogue ----
    const bool l2 = a.l2_out != nullptr;
    double* const stats = a.stats_out ? a.stats_out + (static_cast<int64_t>(my_seg) * RT_STAT_SLOTS +
                                                       blockIdx.x % RT_STAT_SLOTS) * 2 * n : nullptr;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int ct = w + 4 * i;
        const int col = ct * 32 + c32;
        const bool col_ok = col < n;
        const float b = (col_ok && a.bias) ? a.bias[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t gr = row0 + lr;
            const float z = acc[i][r] + b;
            acc[i][r] = z;
            const bool ok = col_ok && gr < m;
            if (ok && a.z_out) a.z_out[gr * n + col] = z;
            if (ok && stats) {
                const float av = act_fwd(a.act, z);
                s1 += av;
                s2 += av * av;
            }
            if (l2) {
                float q = ok ? z * z : 0.f;
#pragma unroll
                for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
                if (c32 == 0) rowpart[ct * FM + lr] = q;
            }
        }
        if (stats) {
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (h == 0 && col_ok) {
                atomicAdd(&stats[col], static_cast<double>(s1));
                atomicAdd(&stats[n + col], static_cast<double>(s2));
            }
        }
    }
    if (l2) {
        __syncthreads();
        const int nt_used = (n + 31) / 32;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int col = (w + 4 * i) * 32 + c32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gr = row0 + lr;
                if (gr < m && col < n) {
                    float ss = 0.f;
                    for (int t = 0; t < nt_used; ++t) ss += rowpart[t * FM + lr];  // fixed order
                    const float nrm = sqrtf(ss);
                    a.l2_out[gr * n + col] = acc[i][r] / fmaxf(nrm, kNormEps);
                    if (col == 0 && a.norms_out) a.norms_out[gr] = nrm;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward 1: dz, dgamma/dbeta, dA = dz·W (+ g_prev / dsrc epilogue)
// ---------------------------------------------------------------------------
// Block = 32 rows. dz (32 x n) lives in LDS; dA = dz·W reads W[n][k] rows
// coalesced along k straight from L2 (the reduction runs over n).
template <int TPWK>  // 32-col dA tiles per wave (k <= 128*TPWK)
__global__ __launch_bounds__(256) void linear_bwd_dz_kernel(rt_linear_bwd_args a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int np = pad8(n), nh = np / 2, ldz = np + 4;
    float* Dz = sm;  // [FM][ldz]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * FM;
    const bool two = a.seg_split > 0;
    const int my_seg = (two && row0 >= a.seg_split) ? 1 : 0;
    const int64_t seg_m = two ? (my_seg == 0 ? a.seg_split : m - a.seg_split) : m;

    // ---- phase A: dz tile ----
    if (a.grad_mode == 0) {
        for (int rr = w * 8; rr < w * 8 + 8; ++rr) {
            const int64_t gr = row0 + rr;
            if (gr < m) {
                float dot = 0.f;
                for (int c = lane; c < n; c += 64) dot += a.l2_out[gr * n + c] * a.dout[gr * n + c];
                dot = wave_sum(dot);
                const float nrm = a.norms[gr];
                const bool big = nrm > kNormEps;
                const float inv = 1.f / (big ? nrm : kNormEps);
                for (int c = lane; c < np; c += 64) {
                    float dz = 0.f;
                    if (c < n) {
                        const float dv = a.dout[gr * n + c];
                        dz = big ? (dv - a.l2_out[gr * n + c] * dot) * inv : dv * inv;
                        a.dz_ws[gr * n + c] = dz;
                    }
                    Dz[rr * ldz + c] = dz;
                }
            } else {
                for (int c = lane; c < np; c += 64) Dz[rr * ldz + c] = 0.f;
            }
        }
    } else {
        // per-column BN-backward coefficients, then a float4 elementwise pass
        float* cA = Dz + FM * ldz;   // γ·invstd (mode 1/2) or 1
        float* cB = cA + np;         // Σg/m
        float* cC = cB + np;         // Σg·x̂/m
        float* cM = cC + np;         // mean
        float* cI = cM + np;         // invstd
        const float inv_m = 1.f / static_cast<float>(seg_m);
        const double* gst = a.g_stats ? a.g_stats + static_cast<int64_t>(my_seg) * RT_STAT_SLOTS * 2 * n : nullptr;
        for (int c = tid; c < np; c += 256) {
            float A = 1.f, Bc = 0.f, C = 0.f, M = 0.f, I = 1.f;
            if (c < n && (a.grad_mode == 1 || a.grad_mode == 2)) {
                I = a.save_invstd[my_seg * n + c];
                M = a.save_mean[my_seg * n + c];
                A = a.bn_gamma[c] * I;
                if (a.grad_mode == 1) {
                    double gs1, gs2;
                    slot_sums(gst, n, c, gs1, gs2);
                    Bc = static_cast<float>(gs1) * inv_m;
                    C = static_cast<float>(gs2) * inv_m;
                }
            }
            cA[c] = A; cB[c] = Bc; cC[c] = C; cM[c] = M; cI[c] = I;
        }
        __syncthreads();
        const int vpr = np / 4;
        const int total = FM * vpr;
        const bool vec = (n % 4) == 0;
        for (int base = tid; base < total; base += 256 * 4) {
            float4 gv[4], zv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                zv[u] = gv[u];
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const int64_t gr = row0 + r;
                    if (gr < m && c < n) {
                        const int64_t off = gr * n + c;
                        if (vec) {
                            gv[u] = *reinterpret_cast<const float4*>(a.g + off);
                            zv[u] = *reinterpret_cast<const float4*>(a.z + off);
                        } else {
                            gv[u].x = a.g[off]; zv[u].x = a.z[off];
                            if (c + 1 < n) { gv[u].y = a.g[off + 1]; zv[u].y = a.z[off + 1]; }
                            if (c + 2 < n) { gv[u].z = a.g[off + 2]; zv[u].z = a.z[off + 2]; }
                            if (c + 3 < n) { gv[u].w = a.g[off + 3]; zv[u].w = a.z[off + 3]; }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                if (e >= total) continue;
                const int r = e / vpr, c = (e - r * vpr) * 4;
                const int64_t gr = row0 + r;
                float dzv[4];
                const float gs[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
                const float zs[4] = {zv[u].x, zv[u].y, zv[u].z, zv[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cc = c + j;
                    float dz = 0.f;
                    if (gr < m && cc < n) {
                        const float xh = (act_fwd(a.act, zs[j]) - cM[cc]) * cI[cc];
                        const float dr = (a.grad_mode == 3) ? gs[j] : cA[cc] * (gs[j] - cB[cc] - xh * cC[cc]);
                        dz = dr * act_bwd(a.act, zs[j]);
                    }
                    dzv[j] = dz;
                }
                *reinterpret_cast<float4*>(Dz + r * ldz + c) = make_float4(dzv[0], dzv[1], dzv[2], dzv[3]);
                if (gr < m && c < n) {
                    const int64_t off = gr * n + c;
                    if (vec) *reinterpret_cast<float4*>(a.dz_ws + off) = make_float4(dzv[0], dzv[1], dzv[2], dzv[3]);
                    else
                        for (int j = 0; j < 4 && c + j < n; ++j) a.dz_ws[off + j] = dzv[j];
                }
            }
        }
    }
    if (blockIdx.x == 0 && (a.grad_mode == 1 || a.grad_mode == 2) && a.dgamma) {
        // dgamma/dbeta of each BN batch (segment), summed like two tower calls' grads
        for (int c = tid; c < n; c += 256) {
            for (int sg = 0; sg < (two ? 2 : 1); ++sg) {
                const double* gs = a.g_stats + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * n;
                double gs1, gs2;
                slot_sums(gs, n, c, gs1, gs2);
                atomicAdd(&a.dgamma[c], static_cast<float>(gs2));  // atomic: concurrent chains of one tower
                atomicAdd(&a.dbeta[c], static_cast<float>(gs1));
            }
        }
    }
    if (!a.g_prev && !a.dsrc) return;
    __syncthreads();

    // ---- phase B: dA = dz · W  (reduction over n, permuted per lane half) ----
    f32x16 acc[TPWK];
#pragma unroll
    for (int i = 0; i < TPWK; ++i) acc[i] = f32x16{};
    const float* dp = Dz + c32 * ldz + h * nh;
    // 8 k-steps per iteration (nh % 16 == 0); next iteration's W loaded during this one's MFMAs
    float wv[TPWK][8], wn[TPWK][8];
    auto load_w = [&](int s, float (&dst)[TPWK][8]) {
#pragma unroll
        for (int i = 0; i < TPWK; ++i) {
            const int kk = (w + 4 * i) * 32 + c32;
            const bool on = (w + 4 * i) * 32 < k && kk < k;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int nn = h * nh + s + j;
                dst[i][j] = (on && nn < n) ? a.w[static_cast<int64_t>(nn) * k + kk] : 0.f;
            }
        }
    };
    load_w(0, wn);
    for (int s = 0; s < nh; s += 8) {
#pragma unroll
        for (int i = 0; i < TPWK; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) wv[i][j] = wn[i][j];
        if (s + 8 < nh) load_w(s + 8, wn);
        float4 av[2];
        av[0] = *reinterpret_cast<const float4*>(dp + s);
        av[1] = *reinterpret_cast<const float4*>(dp + s + 4);
#pragma unroll
        for (int i = 0; i < TPWK; ++i) {
            if ((w + 4 * i) * 32 >= k) continue;  // wave-uniform
            acc[i] = mfma(av[0].x, wv[i][0], acc[i]);
            acc[i] = mfma(av[0].y, wv[i][1], acc[i]);
            acc[i] = mfma(av[0].z, wv[i][2], acc[i]);
            acc[i] = mfma(av[0].w, wv[i][3], acc[i]);
            acc[i] = mfma(av[1].x, wv[i][4], acc[i]);
            acc[i] = mfma(av[1].y, wv[i][5], acc[i]);
            acc[i] = mfma(av[1].z, wv[i][6], acc[i]);
            acc[i] = mfma(av[1].w, wv[i][7], acc[i]);
        }
    }
    const float pscale = a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f;
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const bool want_stats = a.g_prev && a.g_prev_stats && (a.prev_mode == 1 || a.prev_mode == 2);
    double* const gps = want_stats ? a.g_prev_stats + (static_cast<int64_t>(my_seg) * RT_STAT_SLOTS +
                                                        blockIdx.x % RT_STAT_SLOTS) * 2 * k : nullptr;
#pragma unroll
    for (int i = 0; i < TPWK; ++i) {
        const int kk = (w + 4 * i) * 32 + c32;
        const bool col_ok = kk < k;
        float s1 = 0.f, s2 = 0.f;
        float pmean = 0.f, pinv = 0.f;
        if (want_stats && col_ok) { pmean = a.prev_mean[my_seg * k + kk]; pinv = a.prev_invstd[my_seg * k + kk]; }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t gr = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (gr < m && col_ok) {
                const float da = acc[i][r];
                if (a.dsrc) a.dsrc[gr * k + kk] = da;
                if (a.g_prev) {
                    float gv = da;
                    if (a.prev_drop_p > 0.f)
                        gv = dropout_keep(pseed, gr, kk, a.prev_drop_p) ? da * pscale : 0.f;
                    a.g_prev[gr * k + kk] = gv;
                    if (want_stats) {
                        const float xh = (act_fwd(a.prev_act, a.src[gr * a.ld_src + kk]) - pmean) * pinv;
                        s1 += gv;
                        s2 += gv * xh;
                    }
                }
            }
        }
        if (want_stats) {
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (h == 0 && col_ok) {
                atomicAdd(&gps[kk], static_cast<double>(s1));
                atomicAdd(&gps[k + kk], static_cast<double>(s2));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward 2: dW[n][k] += Σ_r dz[r][n] · A[r][k] (+ dbias[n] += Σ_r dz[r][n]),
// M split over blockIdx.z
// ---------------------------------------------------------------------------
// Every wave owns a 64(n) x 32·KT(k) tile (2·KT independent 32x32 accumulators)
// over its own contiguous slice of the block's rows, so the main loop has no
// barrier: each k-step (2 rows) a lane loads dz[r][n0+c32], dz[r][n0+32+c32]
// and A[r][k0+32j+c32] straight from L2/HBM (128 B per half-wave), groups of
// U k-steps are double-buffered in registers (the next group's loads fly
// during the current group's MFMAs), and the A prologue (act → BN affine →
// dropout) runs on registers with per-lane column constants. The 4 waves'
// tiles are summed through LDS and added to dW with one fp32 atomic per
// element per block (<= 32 splits, see the host).
//   PRO: 0 raw A, 1 piecewise-linear act, 2 same + dropout, 3 generic act.
constexpr int DW_N = 64;      // n per block/wave
constexpr int DW_SEG = 2048;  // rows whose gather ids are staged in LDS at a time
constexpr int DW_U = 4;       // k-steps (2 rows each) per register group

template <int PRO>
__device__ __forceinline__ float pro_col(const Pro& p, float slope, int64_t r, int c, float sc, float sh, float v) {
    if constexpr (PRO == 0) {
        return v;
    } else {
        if constexpr (PRO == 3) v = act_fwd(p.act, v);
        else v = act_pwl(slope, v);
        v = __builtin_fmaf(v, sc, sh);
        if constexpr (PRO == 2) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
        if constexpr (PRO == 3) {
            if (p.drop_p > 0.f) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
        }
        return v;
    }
}

template <int KT, int PRO>
__global__ __launch_bounds__(256) void linear_bwd_dw_kernel(rt_linear_bwd_args a, int64_t rows_per_split) {
    constexpr int NT = 2, U = DW_U;
    constexpr int NV = NT * KT * 16;  // accumulator registers per lane
    __shared__ int srow[DW_SEG];
    __shared__ float red[4][NV][64];
    __shared__ float bred[4][DW_N];
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int n0 = blockIdx.x * DW_N, k0 = blockIdx.y * (32 * KT);
    const int64_t r_begin = static_cast<int64_t>(blockIdx.z) * rows_per_split;
    const int64_t r_end = (r_begin + rows_per_split) < m ? (r_begin + rows_per_split) : m;

    int gn[NT], gk[KT];
    bool n_ok[NT], k_ok[KT];
    // BN affine of the previous block per column, per row segment (two BN batches)
    float sc[2][KT], sh[2][KT];
    const bool two = a.seg_split > 0;
#pragma unroll
    for (int i = 0; i < NT; ++i) { gn[i] = n0 + 32 * i + c32; n_ok[i] = gn[i] < n; }
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        gk[j] = k0 + 32 * j + c32;
        k_ok[j] = gk[j] < k;
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
            sc[sg][j] = 1.f; sh[sg][j] = 0.f;
            const int so = two ? sg * k : 0;
            if ((a.prev_mode == 1 || a.prev_mode == 2) && k_ok[j])
                bn_affine(a.prev_gamma[gk[j]], a.prev_beta[gk[j]], a.prev_mean[so + gk[j]], a.prev_invstd[so + gk[j]],
                          sc[sg][j], sh[sg][j]);
        }
    }
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.prev_drop_p, a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f,
                  pseed, nullptr, nullptr};
    const float slope = act_slope(a.prev_act);
    const bool do_bias = a.dbias != nullptr && blockIdx.y == 0;
    const bool gather = a.ids != nullptr;

    f32x16 acc[NT][KT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < KT; ++j) acc[i][j] = f32x16{};
    float bsum[NT] = {};

    float dA[U][NT], xA[U][KT], dB[U][NT], xB[U][KT];
    int64_t seg0 = 0;
    auto load = [&](float (&d)[U][NT], float (&x)[U][KT], int64_t g, int64_t we) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = g + 2 * u + h;
            const bool rv = r < we;
            int64_t sr = r;
            if (gather) sr = rv ? srow[r - seg0] : -1;
#pragma unroll
            for (int i = 0; i < NT; ++i) d[u][i] = (rv && n_ok[i]) ? a.dz_ws[r * n + gn[i]] : 0.f;
#pragma unroll
            for (int j = 0; j < KT; ++j) x[u][j] = (rv && sr >= 0 && k_ok[j]) ? a.src[sr * a.ld_src + gk[j]] : 0.f;
        }
    };
    auto compute = [&](float (&d)[U][NT], float (&x)[U][KT], int64_t g) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = g + 2 * u + h;
#pragma unroll
            for (int j = 0; j < KT; ++j) {
                const int sg = (two && r >= a.seg_split) ? 1 : 0;
                const float xa = pro_col<PRO>(pro, slope, r, gk[j], sg ? sc[1][j] : sc[0][j], sg ? sh[1][j] : sh[0][j],
                                              x[u][j]);
#pragma unroll
                for (int i = 0; i < NT; ++i) acc[i][j] = mfma(d[u][i], xa, acc[i][j]);
            }
            if (do_bias) {
#pragma unroll
                for (int i = 0; i < NT; ++i) bsum[i] += d[u][i];
            }
        }
    };

    for (seg0 = r_begin; seg0 < r_end; seg0 += DW_SEG) {
        const int64_t seg1 = (seg0 + DW_SEG) < r_end ? (seg0 + DW_SEG) : r_end;
        if (gather) {
            __syncthreads();
            for (int t = tid; t < seg1 - seg0; t += 256) {
                const int64_t id = a.ids[seg0 + t];
                srow[t] = (id < 0 || id >= a.src_rows) ? -1 : static_cast<int>(id);
            }
            __syncthreads();
        }
        // this wave's contiguous slice of the segment (multiple of 2U rows)
        const int64_t len = seg1 - seg0;
        const int64_t per = ((len + 3) / 4 + 2 * U - 1) / (2 * U) * (2 * U);
        const int64_t wb = seg0 + w * per;
        const int64_t we = (wb + per) < seg1 ? (wb + per) : seg1;
        if (wb >= we) continue;
        load(dA, xA, wb, we);
        for (int64_t g = wb; g < we; g += 4 * U) {
            if (g + 2 * U < we) load(dB, xB, g + 2 * U, we);
            compute(dA, xA, g);
            if (g + 2 * U >= we) break;
            if (g + 4 * U < we) load(dA, xA, g + 4 * U, we);
            compute(dB, xB, g + 2 * U);
        }
    }

    // ---- sum the 4 waves' tiles through LDS, one atomic per element ----
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < KT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[w][(i * KT + j) * 16 + r][lane] = acc[i][j][r];
    if (do_bias) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const float t = bsum[i] + __shfl_xor(bsum[i], 32, 64);
            if (h == 0) bred[w][32 * i + c32] = t;
        }
    }
    __syncthreads();
    for (int p = tid; p < NV * 64; p += 256) {
        const int v = p >> 6, l = p & 63;
        const float t = red[0][v][l] + red[1][v][l] + red[2][v][l] + red[3][v][l];
        const int i = v / (KT * 16), j = (v / 16) % KT, rr = v & 15;
        const int on = n0 + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * (l >> 5);
        const int ok = k0 + 32 * j + (l & 31);
        if (on < n && ok < k) atomicAdd(&a.dw[static_cast<int64_t>(on) * k + ok], t);
    }
    if (do_bias && tid < DW_N) {
        const int col = n0 + tid;
        if (col < n) atomicAdd(&a.dbias[col], bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid]);
    }
}

}  // namespace mlp
}  // namespace rt

using namespace rt;

// allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); set once per kernel
template <typename K>
static void allow_lds(K kernel, size_t bytes) {
    static size_t set = 0;
    if (bytes > set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(bytes));
        set = bytes;
    }
}

extern "C" int rt_linear_fwd_f32(const rt_linear_fwd_args* args, void* stream) {
    if (!args) return RT_ERR_INVALID;
    const rt_linear_fwd_args& a = *args;
    if (a.m < 0 || a.k <= 0 || a.n <= 0 || !a.src || !a.w || a.ld_src < a.k) return RT_ERR_INVALID;
    if (a.n > 512 || a.k > 8192) return RT_ERR_UNSUPPORTED;
    if (a.prev_mode < 0 || a.prev_mode > 3) return RT_ERR_INVALID;
    if (a.seg_split < 0 || (a.seg_split > 0 && (a.seg_split >= a.m || a.seg_split % mlp::FM != 0)))
        return RT_ERR_INVALID;
    if (a.prev_mode == 1 && (!a.prev_stats || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.prev_mode == 2 && (!a.running_mean || !a.running_var || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.m == 0) return RT_OK;
    const int tpw = a.n <= 128 ? 1 : a.n <= 256 ? 2 : 4;
    const int kp = mlp::pad8(a.k);
    const size_t lds = (2 * kp + mlp::FM * (kp + 4) + 4 * tpw * mlp::FM) * sizeof(float) +
                       mlp::FM * sizeof(int64_t) + 16;
    if (lds > 160 * 1024) return RT_ERR_UNSUPPORTED;
    const bool kvec = (a.k % 4) == 0 && (reinterpret_cast<uintptr_t>(a.w) & 15) == 0;
    const dim3 grid(static_cast<unsigned>((a.m + mlp::FM - 1) / mlp::FM));
    hipStream_t st = as_stream(stream);
#define RT_FWD(T, V)                                                                              \
    do {                                                                                          \
        allow_lds(mlp::linear_fwd_kernel<T, V>, lds);                                             \
        hipLaunchKernelGGL((mlp::linear_fwd_kernel<T, V>), grid, dim3(256), lds, st, a);          \
    } while (0)
    if (kvec) {
        if (tpw == 1) RT_FWD(1, true); else if (tpw == 2) RT_FWD(2, true); else RT_FWD(4, true);
    } else {
        if (tpw == 1) RT_FWD(1, false); else if (tpw == 2) RT_FWD(2, false); else RT_FWD(4, false);
    }
#undef RT_FWD
    return check_launch("linear_fwd_kernel");
}

static int validate_bwd(const rt_linear_bwd_args* args) {
    if (!args) return RT_ERR_INVALID;
    const rt_linear_bwd_args& a = *args;
    if (a.m < 0 || a.k <= 0 || a.n <= 0 || !a.w || !a.dw || !a.dz_ws || !a.src || a.ld_src < a.k)
        return RT_ERR_INVALID;
    const bool need_da = a.g_prev || a.dsrc;
    if (a.n > 2048 || (need_da && a.k > 512)) return RT_ERR_UNSUPPORTED;
    if (a.grad_mode == 0 && (!a.dout || !a.l2_out || !a.norms)) return RT_ERR_INVALID;
    if (a.grad_mode >= 1 && a.grad_mode <= 3 && (!a.g || !a.z)) return RT_ERR_INVALID;
    if ((a.grad_mode == 1 || a.grad_mode == 2) && (!a.g_stats || !a.save_mean || !a.save_invstd || !a.bn_gamma))
        return RT_ERR_INVALID;
    if (a.grad_mode < 0 || a.grad_mode > 3) return RT_ERR_INVALID;
    if (a.seg_split < 0 || (a.seg_split > 0 && (a.seg_split >= a.m || a.seg_split % mlp::FM != 0)))
        return RT_ERR_INVALID;
    if ((a.prev_mode == 1 || a.prev_mode == 2) &&
        (!a.prev_mean || !a.prev_invstd || !a.prev_gamma || !a.prev_beta))
        return RT_ERR_INVALID;
    return RT_OK;
}

extern "C" int rt_linear_bwd_dz_f32(const rt_linear_bwd_args* args, void* stream) {
    const int v = validate_bwd(args);
    if (v) return v;
    const rt_linear_bwd_args& a = *args;
    if (a.m == 0) return RT_OK;
    hipStream_t st = as_stream(stream);
    const bool need_da = a.g_prev || a.dsrc;
    const int tpwk = !need_da ? 1 : a.k <= 128 ? 1 : a.k <= 256 ? 2 : 4;
    const int np = mlp::pad8(a.n);
    const size_t lds = (static_cast<size_t>(mlp::FM) * (np + 4) + 5 * static_cast<size_t>(np)) * sizeof(float) + 16;
    const dim3 grid(static_cast<unsigned>((a.m + mlp::FM - 1) / mlp::FM));
    switch (tpwk) {
        case 1: allow_lds(mlp::linear_bwd_dz_kernel<1>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<1>, grid, dim3(256), lds, st, a); break;
        case 2: allow_lds(mlp::linear_bwd_dz_kernel<2>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<2>, grid, dim3(256), lds, st, a); break;
        default: allow_lds(mlp::linear_bwd_dz_kernel<4>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<4>, grid, dim3(256), lds, st, a); break;
    }
    return check_launch("linear_bwd_dz_kernel");
}

extern "C" int rt_linear_bwd_dw_f32(const rt_linear_bwd_args* args, void* stream) {
    const int v = validate_bwd(args);
    if (v) return v;
    const rt_linear_bwd_args& a = *args;
    if (a.m == 0) return RT_OK;
    hipStream_t st = as_stream(stream);
    const int kt = a.k <= 32 ? 1 : 2;
    const int tn = (a.n + mlp::DW_N - 1) / mlp::DW_N;
    const int tk = (a.k + 32 * kt - 1) / (32 * kt);
    // ~512 blocks (2 per CU), >= 64 rows per block, <= 32 splits per tile
    int64_t splits = (512 + tn * tk - 1) / (tn * tk);
    const int64_t max_splits = (a.m + 63) / 64;
    if (splits > max_splits) splits = max_splits;
    if (splits > 32) splits = 32;
    if (splits < 1) splits = 1;
    int64_t rps = (a.m + splits - 1) / splits;
    rps = (rps + 63) / 64 * 64;
    splits = (a.m + rps - 1) / rps;
    const dim3 grid(static_cast<unsigned>(tn), static_cast<unsigned>(tk), static_cast<unsigned>(splits));
    int pro = 0;
    if (a.prev_mode != 0)
        pro = !act_is_piecewise_linear(a.prev_act) ? 3 : (a.prev_drop_p > 0.f ? 2 : 1);
#define RT_DW(KT, P) hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<KT, P>), grid, dim3(256), 0, st, a, rps)
    if (kt == 1) {
        switch (pro) { case 0: RT_DW(1, 0); break; case 1: RT_DW(1, 1); break; case 2: RT_DW(1, 2); break; default: RT_DW(1, 3); }
    } else {
        switch (pro) { case 0: RT_DW(2, 0); break; case 1: RT_DW(2, 1); break; case 2: RT_DW(2, 2); break; default: RT_DW(2, 3); }
    }
#undef RT_DW
    return check_launch("linear_bwd_dw_kernel");
}

extern "C" int rt_linear_bwd_f32(const rt_linear_bwd_args* args, void* stream) {
    const int rc = rt_linear_bwd_dz_f32(args, stream);
    return rc ? rc : rt_linear_bwd_dw_f32(args, stream);
}
