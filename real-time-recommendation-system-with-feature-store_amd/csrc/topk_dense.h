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
//    Block = 4 waves, tile 128 queries x 64 items, d streamed in 16-wide
//    chunks (register-prefetched one chunk ahead, LDS double buffer of 30 KB:
//    5 blocks per CU); wave w owns query rows 32w..32w+31 and both 32-item
//    column tiles.
// 2. dense_select_kernel: one wave per query over its S row (<= 64 score keys
//    per lane in registers; ties resolved on the composite key (score key <<
//    32 | ~id): score desc, id asc, Faiss's order). The k-th largest of the 64 lane maxima is
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
constexpr int kKC = 16;             // d per LDS chunk (double-buffered: 30 KB per block, 5 blocks per CU)
constexpr int kLS = kKC + 4;        // LDS row stride (floats): 80 B, conflict-free b128 fragment reads
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
    // staging: a chunk is 128 query rows + 64 item rows of 16 floats = 4 float4
    // per row; thread t stages float4 (t % 4) of query rows t / 4 + 64 i and
    // of item row t / 4
    const int c4 = tid & 3, r0 = tid >> 2;
    float4 pq[2], px;
    auto load = [&](int kc) {
        const int dd = kc + 4 * c4;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int64_t q = q0 + r0 + 64 * i;
            pq[i] = (q < nq && dd < d) ? *reinterpret_cast<const float4*>(Q + q * d + dd) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const int64_t x = x0 + r0;
        px = (x < nx && dd < d) ? *reinterpret_cast<const float4*>(X + x * d + dd) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    // [even d | odd d] within the chunk: element 2s + h of the chunk lands at
    // h * kKC/2 + s
    auto store = [&](int b) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            float* row = &Ql[b][(r0 + 64 * i) * kLS];
            *reinterpret_cast<float2*>(row + 2 * c4) = make_float2(pq[i].x, pq[i].z);
            *reinterpret_cast<float2*>(row + kKC / 2 + 2 * c4) = make_float2(pq[i].y, pq[i].w);
        }
        float* row = &Xl[b][r0 * kLS];
        *reinterpret_cast<float2*>(row + 2 * c4) = make_float2(px.x, px.z);
        *reinterpret_cast<float2*>(row + kKC / 2 + 2 * c4) = make_float2(px.y, px.w);
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
        // k-steps of this chunk inside d: 8, or 4 in a last half chunk (d % 8 == 0)
        const int steps = (d - c * kKC) >= kKC ? kKC / 2 : (d - c * kKC) / 2;
#pragma unroll
        for (int s = 0; s < kKC / 2; s += 4) {
            if (s < steps) {
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

// one wave per query; NPL float4 loads per lane (nx <= 256 * NPL). Keys are
// held as 32-bit score keys (okey; 0 = empty); the id of key e of a lane is
// 256·(e/4) + 4·lane + e%4, so the composite (score desc, id asc) key is
// formed only where the radix select needs it.
template <int NPL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void dense_select_kernel(const float* __restrict__ S, int64_t ld, int64_t nq,
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
    uint32_t key[E];
    uint32_t mx = 0u;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int64_t x = 256 * i + 4 * lane;
        const float4 v = x < nx ? *reinterpret_cast<const float4*>(row + x) : make_float4(0.f, 0.f, 0.f, 0.f);
        const uint32_t xb = (ex && x < nx) ? (ex[x >> 5] >> (x & 31)) & 0xFu : 0u;
        const float sv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ok = x + j < nx && !((xb >> j) & 1u);
            key[4 * i + j] = ok ? v2::okey(sv[j]) : 0u;
            mx = key[4 * i + j] > mx ? key[4 * i + j] : mx;
        }
    }
    auto id_of = [&](int e) { return static_cast<uint32_t>(256 * (e >> 2) + 4 * lane + (e & 3)); };
    // k-th largest lane maximum: a bitonic sort of the 64 lane maxima (descending)
    uint32_t t = mx;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int st = size >> 1; st > 0; st >>= 1) {
            const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(t), st, 64));
            const bool lower = (lane & st) == 0;
            const bool desc = (lane & size) == 0;
            t = (lower == desc) ? (o > t ? o : t) : (o < t ? o : t);
        }
    }
    // ties at the bound are kept (a superset of the top k)
    const uint32_t kt = k <= 64 ? static_cast<uint32_t>(__shfl(static_cast<int>(t), k - 1, 64)) : 0u;
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) cnt += (key[e] != 0u && key[e] >= kt) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    // collect: each lane's passing keys as a bit mask (bit e = key e), then a
    // wave-uniform loop that runs max-popcount times (1-3 on a typical row),
    // each lane appending its lowest passing key
    Cand* keep = keep_all[w];
    int m = 0;
    auto collect = [&](uint64_t pm) {
        while (__ballot(pm != 0ull)) {
            const bool has = pm != 0ull;
            const uint64_t bm = __ballot(has);
            const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                    static_cast<uint32_t>(bm >> 32),
                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
            if (has) {
                const int e = __builtin_ctzll(pm);
                pm &= pm - 1ull;
                const uint32_t id = id_of(e);
                if (pos < v4::kFinishCap) keep[pos] = Cand{row[id], id};  // the raw score (okey folds -0.0)
            }
            m += __popcll(bm);
        }
    };
    if (cnt <= v4::kFinishCap) {
        uint64_t pm = 0ull;
#pragma unroll
        for (int e = 0; e < E; ++e) pm |= static_cast<uint64_t>(key[e] != 0u && key[e] >= kt) << e;
        collect(pm);
    } else {
        // many keys at or above the bound (skewed rows, ties, k > 64): radix
        // select on the composite key first
        uint64_t hi = 0ull, lo = ~0ull;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (key[e]) {
                const uint64_t c = (static_cast<uint64_t>(key[e]) << 32) | static_cast<uint32_t>(~id_of(e));
                hi = c > hi ? c : hi;
                lo = c < lo ? c : lo;
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
        uint64_t prefix = hi & v4::prefix_mask(shift);
        int kept = cnt;
        auto eachr = [&](auto&& fn) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (key[e]) fn((static_cast<uint64_t>(key[e]) << 32) | static_cast<uint32_t>(~id_of(e)));
        };
        v4::radix_prefix(eachr, k, v4::kFinishCap, hist_all[w], prefix, shift, kept);
        const uint64_t pmask = v4::prefix_mask(shift);
        uint64_t pm = 0ull;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint64_t c = (static_cast<uint64_t>(key[e]) << 32) | static_cast<uint32_t>(~id_of(e));
            pm |= static_cast<uint64_t>(key[e] != 0u && (c & pmask) >= prefix) << e;
        }
        collect(pm);
    }
    if (m > v4::kFinishCap) m = v4::kFinishCap;  // cannot happen: the bound / prefix limits it
    wave_lds_sync();
    if (m <= 64 && k <= 64) v4::finish_sort<1>(keep, m, k, out_s + q * k, out_i + q * k, id_offset);
    else v4::finish_sort<2>(keep, m, k, out_s + q * k, out_i + q * k, id_offset);
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
