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
// dbias + dA = dz·W with the previous block's dropout/BN-stat epilogue,
// (2) dW = dzᵀ·A over M split across blocks, A recomputed by the same prologue.
#include "rt_common.h"

namespace rt {
namespace mlp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64;        // rows per block (forward, backward-1)
constexpr int KC = 32;        // reduction chunk staged in LDS
constexpr int LDK = KC + 1;   // odd stride: conflict-free ds_read_b32 fragment reads
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

__device__ __forceinline__ void bn_affine(float gamma, float beta, float mean, float invstd, float& scale,
                                          float& shift) {
    scale = gamma * invstd;
    shift = __builtin_fmaf(-mean, scale, beta);
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int TPW>  // 32x32 output tiles per wave; padded width NP = 64*TPW
__global__ __launch_bounds__(256) void linear_fwd_kernel(rt_linear_fwd_args a) {
    constexpr int NP = 64 * TPW;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int kpad = (a.k + KC - 1) / KC * KC;
    float* scale = sm;                       // [kpad]
    float* shift = scale + kpad;             // [kpad]
    float* As = shift + kpad;                // [BM][LDK]
    float* Ws = As + BM * LDK;               // [NP][LDK]
    float* rowpart = Ws + NP * LDK;          // [NP/32][BM] per column-tile row sums (l2)
    int64_t* srow = reinterpret_cast<int64_t*>(rowpart + (NP / 32) * BM);  // [BM]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    const int k = a.k, n = a.n;
    const int64_t m = a.m;

    // ---- prologue setup: BatchNorm affine of the previous block ----
    if (a.prev_mode == 1 || a.prev_mode == 2) {
        for (int c = tid; c < k; c += 256) {
            float mean, invstd, var_f = 0.f;
            if (a.prev_mode == 1) {
                const double md = a.prev_stats[c] / static_cast<double>(m);
                double vd = a.prev_stats[k + c] / static_cast<double>(m) - md * md;
                vd = vd > 0.0 ? vd : 0.0;
                mean = static_cast<float>(md);
                invstd = static_cast<float>(1.0 / sqrt(vd + static_cast<double>(a.bn_eps)));
                var_f = static_cast<float>(m > 1 ? vd * static_cast<double>(m) / static_cast<double>(m - 1) : vd);
            } else {
                mean = a.running_mean[c];
                invstd = static_cast<float>(1.0 / sqrt(static_cast<double>(a.running_var[c]) + a.bn_eps));
            }
            bn_affine(a.bn_gamma[c], a.bn_beta[c], mean, invstd, scale[c], shift[c]);
            if (blockIdx.x == 0) {
                if (a.save_mean) a.save_mean[c] = mean;
                if (a.save_invstd) a.save_invstd[c] = invstd;
                if (a.prev_mode == 1 && a.running_mean) {
                    const float mo = a.bn_momentum;
                    a.running_mean[c] = (1.f - mo) * a.running_mean[c] + mo * mean;
                    a.running_var[c] = (1.f - mo) * a.running_var[c] + mo * var_f;
                }
            }
        }
    }
    for (int r = tid; r < BM; r += 256) {
        const int64_t gr = row0 + r;
        int64_t sr = -1;
        if (gr < m) {
            sr = a.ids ? a.ids[gr] : gr;
            if (sr < 0 || sr >= a.src_rows) sr = -1;
        }
        srow[r] = sr;
    }
    const uint64_t seed = a.drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.drop_p, a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f, seed,
                  scale, shift};

    f32x16 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x16{};
    const int rt = w & 1;
    for (int k0 = 0; k0 < k; k0 += KC) {
        __syncthreads();
        for (int e = tid; e < BM * KC; e += 256) {
            const int r = e / KC, c = e % KC;
            const int gc = k0 + c;
            float v = 0.f;
            const int64_t sr = srow[r];
            if (sr >= 0 && gc < k) v = pro_apply(pro, row0 + r, gc, a.src[sr * a.ld_src + gc]);
            As[r * LDK + c] = v;
        }
        for (int e = tid; e < NP * KC; e += 256) {
            const int nn = e / KC, c = e % KC;
            const int gc = k0 + c;
            Ws[nn * LDK + c] = (nn < n && gc < k) ? a.w[static_cast<int64_t>(nn) * k + gc] : 0.f;
        }
        __syncthreads();
        const float* ap = As + (rt * 32 + c32) * LDK + h;
#pragma unroll 4
        for (int s = 0; s < KC / 2; ++s) {
            const float av = ap[2 * s];
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const int ct = (w >> 1) + 2 * i;
                acc[i] = mfma(av, Ws[(ct * 32 + c32) * LDK + 2 * s + h], acc[i]);
            }
        }
    }

    // ---- epilogue ----
    const bool l2 = a.l2_out != nullptr;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int col = ((w >> 1) + 2 * i) * 32 + c32;
        const bool col_ok = col < n;
        const float b = (col_ok && a.bias) ? a.bias[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lr = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t gr = row0 + lr;
            const float z = acc[i][r] + b;
            acc[i][r] = z;
            const bool ok = col_ok && gr < m;
            if (ok && a.z_out) a.z_out[gr * n + col] = z;
            if (ok && a.stats_out) {
                const float av = act_fwd(a.act, z);
                s1 += av;
                s2 += av * av;
            }
            if (l2) {
                float q = ok ? z * z : 0.f;
#pragma unroll
                for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
                if (c32 == 0) rowpart[((w >> 1) + 2 * i) * BM + lr] = q;
            }
        }
        if (a.stats_out) {
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (h == 0 && col_ok) {
                atomicAdd(&a.stats_out[col], static_cast<double>(s1));
                atomicAdd(&a.stats_out[n + col], static_cast<double>(s2));
            }
        }
    }
    if (l2) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int col = ((w >> 1) + 2 * i) * 32 + c32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gr = row0 + lr;
                if (gr < m && col < n) {
                    float ss = 0.f;
                    for (int t = 0; t < NP / 32; ++t) ss += rowpart[t * BM + lr];  // fixed order
                    const float nrm = sqrtf(ss);
                    a.l2_out[gr * n + col] = acc[i][r] / fmaxf(nrm, kNormEps);
                    if (col == 0 && a.norms_out) a.norms_out[gr] = nrm;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward 1: dz, dbias, dgamma/dbeta, dA = dz·W (+ g_prev / dsrc epilogue)
// ---------------------------------------------------------------------------
template <int TPWK>  // dA output tiles per wave; padded k KP = 64*TPWK
__global__ __launch_bounds__(256) void linear_bwd_dz_kernel(rt_linear_bwd_args a) {
    constexpr int KP = 64 * TPWK;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int npad = (n + KC - 1) / KC * KC;
    const int ldz = npad + 1;
    float* Dz = sm;                       // [BM][ldz]
    float* Wt = Dz + BM * ldz;            // [KP][LDK]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;

    // ---- phase A: dz tile ----
    if (a.grad_mode == 0) {
        for (int rr = w * 16; rr < w * 16 + 16; ++rr) {
            const int64_t gr = row0 + rr;
            if (gr < m) {
                float dot = 0.f;
                for (int c = lane; c < n; c += 64) dot += a.l2_out[gr * n + c] * a.dout[gr * n + c];
                dot = wave_sum(dot);
                const float nrm = a.norms[gr];
                const bool big = nrm > kNormEps;
                const float inv = 1.f / (big ? nrm : kNormEps);
                for (int c = lane; c < npad; c += 64) {
                    float dz = 0.f;
                    if (c < n) {
                        const float dv = a.dout[gr * n + c];
                        dz = big ? (dv - a.l2_out[gr * n + c] * dot) * inv : dv * inv;
                        a.dz_ws[gr * n + c] = dz;
                    }
                    Dz[rr * ldz + c] = dz;
                }
            } else {
                for (int c = lane; c < npad; c += 64) Dz[rr * ldz + c] = 0.f;
            }
        }
    } else {
        const float inv_m = 1.f / static_cast<float>(m);
        for (int e = tid; e < BM * npad; e += 256) {
            const int r = e / npad, c = e % npad;
            const int64_t gr = row0 + r;
            float dz = 0.f;
            if (gr < m && c < n) {
                const float gv = a.g[gr * n + c];
                const float zv = a.z[gr * n + c];
                float dr;
                if (a.grad_mode == 1) {
                    const float mean = a.save_mean[c], invstd = a.save_invstd[c];
                    const float xh = (act_fwd(a.act, zv) - mean) * invstd;
                    const float sg = static_cast<float>(a.g_stats[c]);
                    const float sgx = static_cast<float>(a.g_stats[n + c]);
                    dr = a.bn_gamma[c] * invstd * (gv - sg * inv_m - xh * sgx * inv_m);
                } else if (a.grad_mode == 2) {
                    dr = a.bn_gamma[c] * a.save_invstd[c] * gv;
                } else {
                    dr = gv;
                }
                dz = dr * act_bwd(a.act, zv);
                a.dz_ws[gr * n + c] = dz;
            }
            Dz[r * ldz + c] = dz;
        }
    }
    __syncthreads();
    for (int c = tid; c < n; c += 256) {
        if (a.dbias) {
            float s = 0.f;
            for (int r = 0; r < BM; ++r) s += Dz[r * ldz + c];
            atomicAdd(&a.dbias[c], s);
        }
        if (blockIdx.x == 0 && (a.grad_mode == 1 || a.grad_mode == 2) && a.dgamma) {
            a.dgamma[c] += static_cast<float>(a.g_stats[n + c]);
            a.dbeta[c] += static_cast<float>(a.g_stats[c]);
        }
    }
    if (!a.g_prev && !a.dsrc) return;

    // ---- phase B: dA = dz · W  (reduction over n) ----
    f32x16 acc[TPWK];
#pragma unroll
    for (int i = 0; i < TPWK; ++i) acc[i] = f32x16{};
    const int rt = w & 1;
    for (int n0 = 0; n0 < npad; n0 += KC) {
        __syncthreads();
        for (int e = tid; e < KP * KC; e += 256) {
            const int kk = e % KP, nn = e / KP;
            const int gn = n0 + nn;
            Wt[kk * LDK + nn] = (kk < k && gn < n) ? a.w[static_cast<int64_t>(gn) * k + kk] : 0.f;
        }
        __syncthreads();
        const float* dp = Dz + (rt * 32 + c32) * ldz + n0 + h;
#pragma unroll 4
        for (int s = 0; s < KC / 2; ++s) {
            const float av = dp[2 * s];
#pragma unroll
            for (int i = 0; i < TPWK; ++i) {
                const int ct = (w >> 1) + 2 * i;
                acc[i] = mfma(av, Wt[(ct * 32 + c32) * LDK + 2 * s + h], acc[i]);
            }
        }
    }
    const float pscale = a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f;
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const bool want_stats = a.g_prev && a.g_prev_stats && (a.prev_mode == 1 || a.prev_mode == 2);
#pragma unroll
    for (int i = 0; i < TPWK; ++i) {
        const int kk = ((w >> 1) + 2 * i) * 32 + c32;
        const bool col_ok = kk < k;
        float s1 = 0.f, s2 = 0.f;
        float pmean = 0.f, pinv = 0.f;
        if (want_stats && col_ok) { pmean = a.prev_mean[kk]; pinv = a.prev_invstd[kk]; }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t gr = row0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
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
                atomicAdd(&a.g_prev_stats[kk], static_cast<double>(s1));
                atomicAdd(&a.g_prev_stats[k + kk], static_cast<double>(s2));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward 2: dW[n][k] += Σ_r dz[r][n] · A[r][k], M split over blockIdx.z
// ---------------------------------------------------------------------------
constexpr int DW_T = 64;   // output tile (n) x (k)
constexpr int DW_R = 32;   // rows per staged chunk
constexpr int DW_LD = DW_R + 1;

__global__ __launch_bounds__(256) void linear_bwd_dw_kernel(rt_linear_bwd_args a, int64_t rows_per_split) {
    __shared__ float DzT[DW_T * DW_LD];
    __shared__ float AT[DW_T * DW_LD];
    __shared__ float scale[DW_T], shift[DW_T];
    __shared__ int64_t srow[DW_R];
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int n0 = blockIdx.x * DW_T, k0 = blockIdx.y * DW_T;
    const int64_t r_begin = static_cast<int64_t>(blockIdx.z) * rows_per_split;
    const int64_t r_end = (r_begin + rows_per_split) < m ? (r_begin + rows_per_split) : m;
    if (a.prev_mode == 1 || a.prev_mode == 2) {
        for (int c = tid; c < DW_T; c += 256) {
            const int gc = k0 + c;
            if (gc < k) bn_affine(a.prev_gamma[gc], a.prev_beta[gc], a.prev_mean[gc], a.prev_invstd[gc], scale[c], shift[c]);
            else { scale[c] = 0.f; shift[c] = 0.f; }
        }
    }
    // scale/shift are indexed by the global column inside pro_apply: offset the base
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.prev_drop_p, a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f,
                  pseed, scale - k0, shift - k0};
    const int wn = w & 1, wk = w >> 1;
    f32x16 acc = f32x16{};
    for (int64_t r0 = r_begin; r0 < r_end; r0 += DW_R) {
        __syncthreads();
        if (tid < DW_R) {
            const int64_t gr = r0 + tid;
            int64_t sr = -1;
            if (gr < r_end) {
                sr = a.ids ? a.ids[gr] : gr;
                if (sr < 0 || sr >= a.src_rows) sr = -1;
            }
            srow[tid] = sr;
        }
        __syncthreads();
        for (int e = tid; e < DW_R * DW_T; e += 256) {
            const int rr = e / DW_T, cc = e % DW_T;
            const int64_t gr = r0 + rr;
            const int gn = n0 + cc, gk = k0 + cc;
            float dz = 0.f, av = 0.f;
            if (gr < r_end) {
                if (gn < n) dz = a.dz_ws[gr * n + gn];
                const int64_t sr = srow[rr];
                if (gk < k && sr >= 0) av = pro_apply(pro, gr, gk, a.src[sr * a.ld_src + gk]);
            }
            DzT[cc * DW_LD + rr] = dz;
            AT[cc * DW_LD + rr] = av;
        }
        __syncthreads();
        const float* dp = DzT + (wn * 32 + c32) * DW_LD + h;
        const float* ap = AT + (wk * 32 + c32) * DW_LD + h;
#pragma unroll
        for (int s = 0; s < DW_R / 2; ++s) acc = mfma(dp[2 * s], ap[2 * s], acc);
    }
    const int gk = k0 + wk * 32 + c32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int gn = n0 + wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gn < n && gk < k) atomicAdd(&a.dw[static_cast<int64_t>(gn) * k + gk], acc[r]);
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
    if (a.n > 512 || a.k > 4096) return RT_ERR_UNSUPPORTED;
    if (a.prev_mode < 0 || a.prev_mode > 3) return RT_ERR_INVALID;
    if (a.prev_mode == 1 && (!a.prev_stats || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.prev_mode == 2 && (!a.running_mean || !a.running_var || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.l2_out && a.n > 512) return RT_ERR_UNSUPPORTED;
    if (a.m == 0) return RT_OK;
    const int tpw = a.n <= 64 ? 1 : a.n <= 128 ? 2 : a.n <= 256 ? 4 : 8;
    const int np = 64 * tpw;
    const int kpad = (a.k + mlp::KC - 1) / mlp::KC * mlp::KC;
    const size_t lds = (2 * kpad + mlp::BM * mlp::LDK + np * mlp::LDK + (np / 32) * mlp::BM) * sizeof(float) +
                       mlp::BM * sizeof(int64_t) + 16;
    if (lds > 160 * 1024) return RT_ERR_UNSUPPORTED;
    const dim3 grid(static_cast<unsigned>((a.m + mlp::BM - 1) / mlp::BM));
    hipStream_t st = as_stream(stream);
    switch (tpw) {
        case 1: allow_lds(mlp::linear_fwd_kernel<1>, lds); hipLaunchKernelGGL(mlp::linear_fwd_kernel<1>, grid, dim3(256), lds, st, a); break;
        case 2: allow_lds(mlp::linear_fwd_kernel<2>, lds); hipLaunchKernelGGL(mlp::linear_fwd_kernel<2>, grid, dim3(256), lds, st, a); break;
        case 4: allow_lds(mlp::linear_fwd_kernel<4>, lds); hipLaunchKernelGGL(mlp::linear_fwd_kernel<4>, grid, dim3(256), lds, st, a); break;
        default: allow_lds(mlp::linear_fwd_kernel<8>, lds); hipLaunchKernelGGL(mlp::linear_fwd_kernel<8>, grid, dim3(256), lds, st, a); break;
    }
    return check_launch("linear_fwd_kernel");
}

extern "C" int rt_linear_bwd_f32(const rt_linear_bwd_args* args, void* stream) {
    if (!args) return RT_ERR_INVALID;
    const rt_linear_bwd_args& a = *args;
    if (a.m < 0 || a.k <= 0 || a.n <= 0 || !a.w || !a.dw || !a.dz_ws || !a.src || a.ld_src < a.k)
        return RT_ERR_INVALID;
    const bool need_da = a.g_prev || a.dsrc;
    if (a.n > 256 || (need_da && a.k > 512)) return RT_ERR_UNSUPPORTED;
    if (a.grad_mode == 0 && (!a.dout || !a.l2_out || !a.norms)) return RT_ERR_INVALID;
    if (a.grad_mode >= 1 && a.grad_mode <= 3 && (!a.g || !a.z)) return RT_ERR_INVALID;
    if ((a.grad_mode == 1 || a.grad_mode == 2) && (!a.g_stats || !a.save_mean || !a.save_invstd || !a.bn_gamma))
        return RT_ERR_INVALID;
    if (a.grad_mode < 0 || a.grad_mode > 3) return RT_ERR_INVALID;
    if ((a.prev_mode == 1 || a.prev_mode == 2) &&
        (!a.prev_mean || !a.prev_invstd || !a.prev_gamma || !a.prev_beta))
        return RT_ERR_INVALID;
    if (a.m == 0) return RT_OK;
    hipStream_t st = as_stream(stream);
    {
        const int tpwk = !need_da ? 1 : a.k <= 64 ? 1 : a.k <= 128 ? 2 : a.k <= 256 ? 4 : 8;
        const int kp = need_da ? 64 * tpwk : 0;
        const int npad = (a.n + mlp::KC - 1) / mlp::KC * mlp::KC;
        const size_t lds = (static_cast<size_t>(mlp::BM) * (npad + 1) + static_cast<size_t>(kp) * mlp::LDK) *
                           sizeof(float);
        if (lds > 160 * 1024) return RT_ERR_UNSUPPORTED;
        const dim3 grid(static_cast<unsigned>((a.m + mlp::BM - 1) / mlp::BM));
        switch (tpwk) {
            case 1: allow_lds(mlp::linear_bwd_dz_kernel<1>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<1>, grid, dim3(256), lds, st, a); break;
            case 2: allow_lds(mlp::linear_bwd_dz_kernel<2>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<2>, grid, dim3(256), lds, st, a); break;
            case 4: allow_lds(mlp::linear_bwd_dz_kernel<4>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<4>, grid, dim3(256), lds, st, a); break;
            default: allow_lds(mlp::linear_bwd_dz_kernel<8>, lds); hipLaunchKernelGGL(mlp::linear_bwd_dz_kernel<8>, grid, dim3(256), lds, st, a); break;
        }
        const int rc = check_launch("linear_bwd_dz_kernel");
        if (rc) return rc;
    }
    {
        const int tn = (a.n + mlp::DW_T - 1) / mlp::DW_T;
        const int tk = (a.k + mlp::DW_T - 1) / mlp::DW_T;
        int64_t splits = (512 + tn * tk - 1) / (tn * tk);
        const int64_t max_splits = (a.m + 63) / 64;
        if (splits > max_splits) splits = max_splits;
        if (splits < 1) splits = 1;
        int64_t rps = (a.m + splits - 1) / splits;
        rps = (rps + mlp::DW_R - 1) / mlp::DW_R * mlp::DW_R;
        splits = (a.m + rps - 1) / rps;
        const dim3 grid(static_cast<unsigned>(tn), static_cast<unsigned>(tk), static_cast<unsigned>(splits));
        hipLaunchKernelGGL(mlp::linear_bwd_dw_kernel, grid, dim3(256), 0, st, a, rps);
        return check_launch("linear_bwd_dw_kernel");
    }
}
