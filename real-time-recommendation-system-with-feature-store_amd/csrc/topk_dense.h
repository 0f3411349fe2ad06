// Flat-IP top-K for SMALL fp32 corpora (nx <= 4096, the C3 serving shape:
// 6,040 users x 3,416 movies, and the MovieLens offline evaluation), as two
// launches instead of one fused scan — faiss.IndexFlatIP.search
// (src/serving/retrieval.py:170-171) and the masked np.dot + argsort of
// scripts/evaluate_model.py:217-232.
//
// 1. dense_scores_kernel: S = Q·Xᵀ for a chunk of queries, a plain fp32 MFMA
//    GEMM (v_mfma_f32_32x32x2_f32, A = query rows, B = item rows) written to a
//    row-major [nq_chunk][ld] slab that stays in the 256 MB Infinity Cache.
//    Every S[q][x] is ONE accumulation chain over d in increasing order
//    (k-step s feeds d = 2s on lane half 0, 2s + 1 on half 1; rows staged in
//    LDS as [even d | odd d] so a ds_read_b128 feeds four k-steps), i.e. the
//    sequential fmaf chain of oracle/flatip.c, bit for bit.
//    Block = 4 waves, tile 128 queries x 64 items, d streamed in 32-wide
//    chunks (register-prefetched one chunk ahead, LDS double buffer); wave w
//    owns query rows 32w..32w+31 and both 32-item column tiles.
// 2. dense_select_kernel: one wave per query over its S row (<= 64 keys per
//    lane in registers, the composite key (score key << 32 | ~id): score
//    desc, id asc, Faiss's order). The k-th largest of the 64 lane maxima is
//    a lower bound of the row's k-th key (k lanes hold a key >= it), so the
//    keys >= it hold the top k; when they are few (<= 128: the usual case)
//    they are sorted at once, otherwise the v4 radix select narrows them
//    first. Scores are written from the slab (the raw float: -0.0 kept).
// The fused register-list kernel (topk_impl.h) spent its time in sorted-list
// inserts beside 64-cycle fp32 MFMAs; here the GEMM runs with no selection
// VALU in its loop and the selection runs with no MFMA beside it.
#pragma once

namespace rt {
namespace topk {
namespace dense {

constexpr int kMaxNx = 4096;       // items per query row the select wave holds (64 lanes x 64)
constexpr int kBQ = 128, kBX = 64;  // GEMM block tile (queries x items)
constexpr int kKC = 32;             // d per LDS chunk
constexpr int kLS = kKC + 4;        // LDS row stride (floats): 144 B
constexpr int64_t kSlabBytes = 256ll << 20;  // S slab per launch (<= the Infinity Cache)

inline int64_t ld_for(int64_t nx) { return (nx + 63) / 64 * 64; }

// queries per launch: the slab fits kSlabBytes, a multiple of the block tile
inline int64_t chunk_for(int64_t nq, int64_t nx) {
    int64_t c = kSlabBytes / (ld_for(nx) * 4);
    c = c / kBQ * kBQ;
    if (c < kBQ) c = kBQ;
    return nq < c ? nq : c;
}

template <int BQ = kBQ>  // a template so the three dtype translation units share one definition
__global__ __launch_bounds__(256) void dense_scores_kernel(const float* __restrict__ Q, int64_t nq,
                                                           const float* __restrict__ X, int64_t nx, int d,
                                                           float* __restrict__ S, int64_t ld) {
    __shared__ __attribute__((aligned(16))) float Ql[2][kBQ * kLS];
    __shared__ __attribute__((aligned(16))) float Xl[2][kBX * kLS];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    const int64_t tiles_x = (nx + kBX - 1) / kBX;
    static_assert(BQ == kBQ, "one tile shape");
    const int64_t q0 = static_cast<int64_t>(blockIdx.x / tiles_x) * kBQ;
    const int64_t x0 = static_cast<int64_t>(blockIdx.x % tiles_x) * kBX;
    // staging: a chunk is 128 query rows + 64 item rows of 32 floats = 8 float4
    // per row; thread t stages float4 (t % 8) of rows t / 8 + 32 i
    const int c4 = tid & 7, r0 = tid >> 3;
    float4 pq[4], px[2];
    auto load = [&](int kc) {
        const int dd = kc + 4 * c4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t q = q0 + r0 + 32 * i;
            pq[i] = (q < nq && dd < d) ? *reinterpret_cast<const float4*>(Q + q * d + dd) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int64_t x = x0 + r0 + 32 * i;
            px[i] = (x < nx && dd < d) ? *reinterpret_cast<const float4*>(X + x * d + dd) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    // [even d | odd d] within the chunk: element 2s + h of the chunk lands at
    // h * kKC/2 + s
    auto store = [&](int b) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float* row = &Ql[b][(r0 + 32 * i) * kLS];
            *reinterpret_cast<float2*>(row + 2 * c4) = make_float2(pq[i].x, pq[i].z);
            *reinterpret_cast<float2*>(row + kKC / 2 + 2 * c4) = make_float2(pq[i].y, pq[i].w);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            float* row = &Xl[b][(r0 + 32 * i) * kLS];
            *reinterpret_cast<float2*>(row + 2 * c4) = make_float2(px[i].x, px[i].z);
            *reinterpret_cast<float2*>(row + kKC / 2 + 2 * c4) = make_float2(px[i].y, px[i].w);
        }
    };
    f32x16 acc0 = f32x16{}, acc1 = f32x16{};
    const int nchunks = (d + kKC - 1) / kKC;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int b = c & 1;
        if (c + 1 < nchunks) load((c + 1) * kKC);
        const float* qa = &Ql[b][(32 * w + col) * kLS + half * (kKC / 2)];
        const float* xa = &Xl[b][col * kLS + half * (kKC / 2)];
        const float* xb = &Xl[b][(32 + col) * kLS + half * (kKC / 2)];
        // k-steps of this chunk that lie inside d (d % 8 == 0: whole groups of 4)
        int steps = (d - c * kKC) / 2;
        steps = steps > kKC / 2 ? kKC / 2 : steps;
        for (int s = 0; s < steps; s += 4) {
            const float4 a = *reinterpret_cast<const float4*>(qa + s);
            const float4 u = *reinterpret_cast<const float4*>(xa + s);
            const float4 v = *reinterpret_cast<const float4*>(xb + s);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, u.x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, v.x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, u.y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, v.y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, u.z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, v.z, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, u.w, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, v.w, acc1, 0, 0, 0);
        }
        if (c + 1 < nchunks) store(b ^ 1);
        __syncthreads();
    }
    // acc[r] at lane (col, half) = S[q0 + 32w + tile_row(r, half)][x0 + 32j + col]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * w + tile_row(r, half);
        if (q < nq) {
            float* srow = S + q * ld + x0 + col;
            srow[0] = acc0[r];    // columns past nx land in the slab's padding (ld >= tiles_x * kBX)
            srow[32] = acc1[r];
        }
    }
}

// one wave per query; NPL float4 loads per lane (nx <= 256 * NPL)
template <int NPL>
__global__ __launch_bounds__(256) void dense_select_kernel(const float* __restrict__ S, int64_t ld, int64_t nq,
                                                           int64_t nx, int k, const uint32_t* __restrict__ excl,
                                                           int64_t excl_words, float* __restrict__ out_s,
                                                           int64_t* __restrict__ out_i, int64_t id_offset) {
    __shared__ __attribute__((aligned(16))) uint32_t hist_all[4][256];
    __shared__ __attribute__((aligned(16))) Cand keep_all[4][v4::kFinishCap];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (q >= nq) return;  // wave-uniform; only wave-level LDS sync below
    const float* row = S + q * ld;
    const uint32_t* ex = excl ? excl + q * excl_words : nullptr;
    constexpr int E = 4 * NPL;
    uint64_t key[E];
    float4 v[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int64_t x = 256 * i + 4 * lane;
        v[i] = x < nx ? *reinterpret_cast<const float4*>(row + x) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint32_t xw[NPL];  // exclusion bits of this lane's 4 items per load (a 4-bit nibble)
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int64_t x = 256 * i + 4 * lane;
        xw[i] = (ex && x < nx) ? (ex[x >> 5] >> (x & 31)) & 0xFu : 0u;
    }
    uint64_t mx = 0ull;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const float sv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t x = 256 * i + 4 * lane + j;
            const bool ok = x < nx && !((xw[i] >> j) & 1u);
            key[4 * i + j] = ok ? ((static_cast<uint64_t>(v2::okey(sv[j])) << 32) | static_cast<uint32_t>(~x)) : 0ull;
            mx = key[4 * i + j] > mx ? key[4 * i + j] : mx;
        }
    }
    // k-th largest lane maximum: a bitonic sort of the 64 lane maxima (descending)
    uint64_t t = mx;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int st = size >> 1; st > 0; st >>= 1) {
            const uint64_t o = __shfl_xor(t, st, 64);
            const bool lower = (lane & st) == 0;        // keeps the larger in a descending run
            const bool desc = (lane & size) == 0 || size == 64;
            const bool take_max = lower == desc;
            t = take_max ? (o > t ? o : t) : (o < t ? o : t);
        }
    }
    const uint64_t kt = k <= 64 ? __shfl(t, k - 1, 64) : 0ull;  // 0: no bound (every non-empty key)
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) cnt += (key[e] != 0ull && key[e] >= kt) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    uint64_t prefix = kt;
    uint64_t pmask = ~0ull;
    if (cnt > v4::kFinishCap) {
        // many keys above the bound (skewed rows, large k): radix select first
        uint64_t hi = 0ull, lo = ~0ull;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (key[e]) {
                hi = key[e] > hi ? key[e] : hi;
                lo = key[e] < lo ? key[e] : lo;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a = __shfl_xor(hi, o, 64), b = __shfl_xor(lo, o, 64);
            hi = a > hi ? a : hi;
            lo = b < lo ? b : lo;
        }
        int shift = 64 - (hi == lo ? 64 : __builtin_clzll(hi ^ lo));
        if (shift < 8) shift = 8;
        uint64_t pre = hi & v4::prefix_mask(shift);
        int kept = cnt;
        auto eachr = [&](auto&& fn) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (key[e]) fn(key[e]);
        };
        v4::radix_prefix(eachr, k, v4::kFinishCap, hist_all[w], pre, shift, kept);
        prefix = pre;
        pmask = v4::prefix_mask(shift);
    }
    Cand* keep = keep_all[w];
    int m = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const bool take = key[e] != 0ull && (key[e] & pmask) >= prefix;
        const uint64_t bm = __ballot(take);
        const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                static_cast<uint32_t>(bm >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
        if (take && pos < v4::kFinishCap) {
            const uint32_t id = ~static_cast<uint32_t>(key[e]);
            keep[pos] = Cand{row[id], id};  // the raw score (okey folds -0.0 onto +0.0)
        }
        m += __popcll(bm);
    }
    if (m > v4::kFinishCap) m = v4::kFinishCap;  // cannot happen: the bound / prefix limits it
    wave_lds_sync();
    v4::finish_sort<2>(keep, m, k, out_s + q * k, out_i + q * k, id_offset);
}

inline bool applies(int64_t nx, int d, int k) { return nx > 0 && nx <= kMaxNx && d % 8 == 0 && d <= 256 && k <= 128; }

inline int launch(const Args& a, float* slab, int64_t ld, hipStream_t st) {
    const int64_t tiles = ((a.nq + kBQ - 1) / kBQ) * ((a.nx + kBX - 1) / kBX);
    hipLaunchKernelGGL(dense_scores_kernel<kBQ>, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, st,
                       reinterpret_cast<const float*>(a.Q), a.nq, reinterpret_cast<const float*>(a.X), a.nx, a.d,
                       slab, ld);
    int rc = check_launch("dense_scores_kernel");
    if (rc) return rc;
    const dim3 grid(static_cast<unsigned>((a.nq + 3) / 4));
    const int npl = static_cast<int>((a.nx + 255) / 256);
#define RT_SEL(N) hipLaunchKernelGGL(dense_select_kernel<N>, grid, dim3(256), 0, st, slab, ld, a.nq, a.nx, a.k, \
                                     a.excl, a.excl_words, a.out_s, a.out_i, a.id_offset)
    if (npl <= 4) RT_SEL(4);
    else if (npl <= 8) RT_SEL(8);
    else RT_SEL(16);
#undef RT_SEL
    return check_launch("dense_select_kernel");
}

}  // namespace dense
}  // namespace topk
}  // namespace rt
