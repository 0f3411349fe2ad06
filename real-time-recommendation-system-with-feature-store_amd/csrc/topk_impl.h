// Brute-force inner-product top-K kernel (Faiss IndexFlatIP equivalent), gfx950.
// Included by topk_{f32,f16,bf16}.hip (one dtype per translation unit).
//
// Replaces faiss.IndexFlatIP.search (src/serving/retrieval.py:96-98,171) and
// the masked np.dot + argsort of scripts/evaluate_model.py:217-232.
//
// * block = 4 waves; wave w owns QS sets of 32 queries. The MFMA is oriented
//   ITEMS × QUERIES (A = item rows from LDS, B = query fragments held in
//   registers for the whole scan), so each lane's accumulator column is ONE
//   query and every A fragment read from LDS feeds QS MFMAs.
// * items stream through LDS in NT-row tiles, register-prefetched one tile
//   ahead; 32x32 MFMA sub-tiles (fp32: v_mfma_f32_32x32x2_f32 — a sequential
//   fmaf chain over d, bit-exact vs oracle/flatip.c; f16/bf16:
//   v_mfma_f32_32x32x16_*).
// * selection, per lane (= per query, per wave half): the 16 scores of a
//   sub-tile are max-reduced and compared with the lane's threshold first, so
//   a sub-tile with no candidate in the whole wave costs ~16 VALU ops; a
//   sorted top-K list (K = 16 or 32 >= k) lives in registers, insertion by K
//   compare-swaps; the two wave halves' lists are merged by a bitonic merge at
//   the end. Ties are broken by id (lower id first), as in Faiss's heap.
// * this register-list kernel serves fp32 with k <= 32 (C3 / serving: the
//   64-cycle fp32 MFMAs of a sub-tile hide the insertion work); 16-bit scans
//   and larger k use the candidate-buffer kernel of topk_v1.h.
#pragma once

#include <float.h>

#include "rt_common.h"
#include "rt_sort.h"

namespace rt {
namespace topk {

constexpr int kWaves = 4;
constexpr int kMaxK = 512;
constexpr int kMaxCap = 1024;
constexpr int64_t kQueryChunk = 1 << 16;  // queries per launch (bounds the workspace)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct Mfma;
template <> struct Mfma<float> {
    static constexpr int kK = 2;      // k per instruction
    typedef float frag;
    __device__ static f32x16 run(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma<__half> {
    static constexpr int kK = 16;
    typedef h8 frag;
    __device__ static f32x16 run(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma<__hip_bfloat16> {
    static constexpr int kK = 16;
    typedef b8 frag;
    __device__ static f32x16 run(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};

template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag frag_from(const T* p) {
    if constexpr (Mfma<T>::kK == 2) {
        return *p;
    } else {
        const uint4 u = *reinterpret_cast<const uint4*>(p);
        return __builtin_bit_cast(typename Mfma<T>::frag, u);
    }
}

// compile-time shape of one instantiation
template <typename T, int S, int MODE>  // MODE = K, the register list length
struct Cfg {
    static constexpr int KK = Mfma<T>::kK;
    static constexpr int DP = S * KK;                                           // padded d
    static constexpr int QREGS = S * static_cast<int>(sizeof(typename Mfma<T>::frag) / 4);  // per query set
    static constexpr int LREGS = 2 * MODE;                                     // register list
    // query sets per wave: fragments + lists within ~128 VGPRs
    static constexpr int QS_RAW = 128 / (QREGS + LREGS);
    static constexpr int QS = QS_RAW >= 4 ? 4 : (QS_RAW >= 2 ? 2 : 1);
    static constexpr int QT = 32 * QS * kWaves;                                // queries per block
    static constexpr int NT = 64;                                              // items per LDS tile
    static constexpr int VEC = 16 / static_cast<int>(sizeof(T));               // elements per 16 B
    static constexpr int LS = DP + VEC;                                        // +16 B pad per row
    static constexpr int TILE_VECS = NT * (DP / VEC);
    static constexpr int LOADS = (TILE_VECS + 255) / 256;
};

struct Plan {
    int64_t chunk;       // queries per launch
    int q_tiles;         // blocks along queries per launch
    int splits;          // blocks along items
    int64_t items_per_split;
    int cap;             // candidate buffer entries per query (v1 kernel), else 0
    size_t cand_bytes, part_bytes;
    int v4;              // 1: the sampled-threshold scan + finish pair (topk_v4.h)
    int v4_joint;        // v4 over > 1 split: one threshold per query from a corpus-wide sample
    size_t fail_bytes;   // v4 joint: per-query flags (union of the split buffers < k)
    int stride, rank;    // v4 sample: every stride-th stage; threshold = rank-th group maximum
    int v4_presample;    // v4 joint: one sample-only scan of every split, then the thresholds (launch_presampled)
    size_t lists_bytes, thr_bytes;  // v4 presampled plan workspaces
    size_t meta_bytes;   // v4 per-(split, query) entry counts
    size_t kth_bytes;    // register-list kernel over > 1 split: the shared per-query k-th keys
    int dense;           // 1: fp32 small corpus, GEMM into a score slab + per-query select (topk_dense.h)
};

struct Args {
    const void* Q; int64_t nq; const void* X; int64_t nx; int d; int k;
    const uint32_t* excl; int64_t excl_words;
    Cand* cand; float* out_s; int64_t* out_i; int64_t id_offset;
    int* meta;
    int* fail;             // v4 joint threshold: per-query rescue flags (nullptr: per-split mode)
    const float* thr_in;   // v4 mode 4: per-query thresholds (a presample's, or a caller's)
    float* lists_out;      // v4 mode 3: [splits][q_pad][32] sampled group maxima per query
    float* v4_lists;       // v4 presampled plan: workspace of the mode-3 lists
    float* v4_thr;         // v4 presampled plan: workspace of the per-query thresholds
    uint32_t* kth_shared;  // register-list kernel, split corpora: per query, the best split k-th score (okey)
};

// order-preserving key of a score (-0 folded onto +0); 0 sorts below every score
__device__ __forceinline__ uint32_t score_key(float s) {
    const uint32_t u = __float_as_uint(s + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float score_of_key(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__device__ __forceinline__ int tile_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// insert (cs, ci) into a sorted (better-first) register list of K entries
template <int K>
__device__ __forceinline__ void list_insert(float (&ls)[K], uint32_t (&li)[K], float cs, uint32_t ci) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const bool b = better(cs, ci, ls[i], li[i]);
        const float ts = ls[i];
        const uint32_t ti = li[i];
        ls[i] = b ? cs : ts;
        li[i] = b ? ci : ti;
        cs = b ? ts : cs;
        ci = b ? ti : ci;
    }
}

// bitonic sort of N (a power of two) register entries of one lane, better first
template <int N>
__device__ __forceinline__ void lane_sort(float (&s)[N], uint32_t (&id)[N]) {
#pragma unroll
    for (int size = 2; size <= N; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if ((i & stride) == 0) {
                    const int j = i | stride;
                    const bool up = (i & size) == 0;
                    if (better(s[j], id[j], s[i], id[i]) == up) {
                        const float ts = s[i];
                        const uint32_t ti = id[i];
                        s[i] = s[j];
                        id[i] = id[j];
                        s[j] = ts;
                        id[j] = ti;
                    }
                }
            }
}

template <typename T, int S, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void flatip_topk_kernel(Args a,
                                                                                       int64_t items_per_split) {
    using M = Mfma<T>;
    using C = Cfg<T, S, K>;
    constexpr int KK = C::KK, QS = C::QS, QT = C::QT, NT = C::NT, LS = C::LS, VEC = C::VEC, DP = C::DP;
    constexpr int TILE_VECS = C::TILE_VECS, LOADS = C::LOADS;
    __shared__ __attribute__((aligned(16))) T tile[NT * LS];

    const T* __restrict__ Q = reinterpret_cast<const T*>(a.Q);
    const T* __restrict__ X = reinterpret_cast<const T*>(a.X);
    const int d = a.d, k = a.k;
    const int64_t nq = a.nq;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    const int64_t qb = static_cast<int64_t>(blockIdx.x) * QT + wave * 32 * QS;  // wave's first query
    const int split = blockIdx.y;
    const int64_t i_begin = static_cast<int64_t>(split) * items_per_split;
    const int64_t i_end = (i_begin + items_per_split) < a.nx ? (i_begin + items_per_split) : a.nx;
    const int row_vecs = d / VEC;

    // ---- query fragments in registers: B[k][query]; per-lane top-K lists ----
    typename M::frag qf[QS][S];
    bool qok[QS];
    const uint32_t* excl[QS];
    float th[QS];
    float ls[QS][K];
    uint32_t li[QS][K];
#pragma unroll
    for (int j = 0; j < QS; ++j) {
        const int64_t q = qb + j * 32 + col;
        qok[j] = q < nq;
        const T* qrow = Q + (qok[j] ? q : 0) * d;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k0 = (KK == 2) ? (2 * s + half) : (16 * s + 8 * half);
            if (qok[j] && k0 < d) qf[j][s] = frag_from<T>(qrow + k0);
            else qf[j][s] = typename M::frag{};
        }
        excl[j] = (a.excl && qok[j]) ? a.excl + q * a.excl_words : nullptr;
        th[j] = qok[j] ? -INFINITY : INFINITY;
#pragma unroll
        for (int i = 0; i < K; ++i) { ls[j][i] = -INFINITY; li[j][i] = kEmptyId; }
    }

    // register prefetch of one tile (rows t0 .. t0+NT-1, zero padded)
    uint4 pre[LOADS];
    auto fetch = [&](int64_t t0) {
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            const int e = tid + l * 256;
            const int r = e / (DP / VEC);
            const int c = e % (DP / VEC);
            const int64_t item = t0 + r;
            pre[l] = make_uint4(0, 0, 0, 0);
            if (e < TILE_VECS && item < i_end && c < row_vecs)
                pre[l] = *reinterpret_cast<const uint4*>(X + item * d + c * VEC);
        }
    };
    fetch(i_begin);

    // k-th of a lane's sorted list (k <= K, runtime): a select chain
    auto kth_of = [&](const float (&l)[K]) {
        float v = l[0];
#pragma unroll
        for (int i = 1; i < K; ++i) v = (i == k - 1) ? l[i] : v;
        return v;
    };
    // cross-split k-th: the value the previous tile's atomic max returned
    // (half-0 lanes; consumed one tile later, so the atomic's latency hides
    // behind a tile of MFMAs)
    uint32_t ret_key[QS];
#pragma unroll
    for (int j = 0; j < QS; ++j) ret_key[j] = 0u;
    for (int64_t t0 = i_begin; t0 < i_end; t0 += NT) {
        __syncthreads();  // previous tile consumed
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            const int e = tid + l * 256;
            if (e < TILE_VECS) {
                const int r = e / (DP / VEC);
                const int c = e % (DP / VEC);
                if constexpr (KK == 2) {
                    // fp32: a row is stored as [even k | odd k] so that the lane
                    // that feeds k-step s (element 2s + half) reads 4 steps in one
                    // ds_read_b128 — the natural k order, unchanged, bit-exact
                    const uint4 v = pre[l];
                    *reinterpret_cast<uint2*>(tile + r * LS + 2 * c) = make_uint2(v.x, v.z);
                    *reinterpret_cast<uint2*>(tile + r * LS + DP / 2 + 2 * c) = make_uint2(v.y, v.w);
                } else {
                    *reinterpret_cast<uint4*>(tile + r * LS + c * VEC) = pre[l];
                }
            }
        }
        __syncthreads();
        if (t0 != i_begin) {
            // Tighten each query's filter (any value <= the final k-th of this
            // split's lists is valid; inserts stay strict >). Own list: its k-th,
            // not its K-th. The partner half (lane ^ 32): its k-th too — its
            // items precede every later item of mine, so an equal later score
            // loses by id. Other splits: their k-th is <= the global k-th, but
            // their ids may be larger than mine, so ties must still enter — one
            // float step below it.
#pragma unroll
            for (int j = 0; j < QS; ++j) {
                float t = kth_of(ls[j]);
                t = fmaxf(t, __shfl_xor(t, 32, 64));
                if (a.kth_shared) {
                    const uint32_t prev = static_cast<uint32_t>(__shfl(static_cast<int>(ret_key[j]), col, 64));
                    const float mine = t;
                    if (prev) t = fmaxf(t, nextafterf(score_of_key(prev), -INFINITY));
                    const int64_t q = qb + j * 32 + col;
                    if (half == 0 && qok[j] && mine > -INFINITY)
                        ret_key[j] = atomicMax(a.kth_shared + q, score_key(mine));
                }
                if (qok[j] && t > th[j]) th[j] = t;
            }
        }
        if (t0 + NT < i_end) fetch(t0 + NT);  // overlaps the MFMA work below
#pragma unroll 1
        for (int rt = 0; rt < NT / 32; ++rt) {
            const int64_t sub0 = t0 + rt * 32;
            if (sub0 >= i_end) break;  // block-uniform
            f32x16 acc[QS];
#pragma unroll
            for (int j = 0; j < QS; ++j) acc[j] = f32x16{};
            if constexpr (KK == 2) {
                // k-steps s..s+3 of this lane: 4 consecutive floats of its half
                const T* arow = tile + (rt * 32 + col) * LS + half * (DP / 2);
#pragma unroll
                for (int s = 0; s < S; s += 4) {
                    const float4 a4 = *reinterpret_cast<const float4*>(arow + s);
#pragma unroll
                    for (int j = 0; j < QS; ++j) {
                        acc[j] = M::run(a4.x, qf[j][s], acc[j]);
                        acc[j] = M::run(a4.y, qf[j][s + 1], acc[j]);
                        acc[j] = M::run(a4.z, qf[j][s + 2], acc[j]);
                        acc[j] = M::run(a4.w, qf[j][s + 3], acc[j]);
                    }
                }
            } else {
                const T* arow = tile + (rt * 32 + col) * LS + 8 * half;
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const typename M::frag af = frag_from<T>(arow + s * KK);
#pragma unroll
                    for (int j = 0; j < QS; ++j) acc[j] = M::run(af, qf[j][s], acc[j]);
                }
            }
            if (sub0 + 32 > i_end) {  // partial last sub-tile: rows past the end never qualify
                const int left = static_cast<int>(i_end - sub0);
#pragma unroll
                for (int j = 0; j < QS; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (tile_row(r, half) >= left) acc[j][r] = -INFINITY;
            }
#pragma unroll
            for (int j = 0; j < QS; ++j) {
                float mx = acc[j][0];
#pragma unroll
                for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[j][r]);
                if (__ballot(mx > th[j]) == 0) continue;  // wave-uniform skip
                const f32x16 aj = acc[j];
                if (t0 == i_begin && rt == 0) {
                    // the split's first sub-tile meets empty lists: one sort of
                    // the lane's 16 rows gives the list 16 in-order inserts
                    // would build (rows that would not insert become empties)
                    float s16[16];
                    uint32_t i16[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t item = static_cast<uint32_t>(sub0 + tile_row(r, half));
                        bool ok = qok[j] && aj[r] > th[j];
                        if (ok && excl[j]) ok = !((excl[j][item >> 5] >> (item & 31)) & 1u);
                        s16[r] = ok ? aj[r] : -INFINITY;
                        i16[r] = ok ? item : kEmptyId;
                    }
                    lane_sort<16>(s16, i16);
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        ls[j][i] = i < 16 ? s16[i < 16 ? i : 0] : -INFINITY;
                        li[j][i] = i < 16 ? i16[i < 16 ? i : 0] : kEmptyId;
                    }
                    if (qok[j]) th[j] = ls[j][K - 1];
                    continue;
                }
                // per-lane pass mask; the wave loops max-popcount times (not 16),
                // each lane taking its passing rows in increasing r (= id) order,
                // the order of the plain r loop, so the lists come out the same
                uint32_t bits = 0u;
#pragma unroll
                for (int r = 0; r < 16; ++r) bits |= (aj[r] > th[j] ? 1u : 0u) << r;
                while (__ballot(bits != 0u)) {
                    if (bits) {
                        const int r = __builtin_ctz(bits);
                        bits &= bits - 1u;
                        float v = aj[0];
#pragma unroll
                        for (int rr = 1; rr < 16; ++rr) v = (r == rr) ? aj[rr] : v;
                        const uint32_t item = static_cast<uint32_t>(sub0 + tile_row(r, half));
                        const bool ex = excl[j] && ((excl[j][item >> 5] >> (item & 31)) & 1u);
                        if (v > th[j] && !ex) {
                            list_insert<K>(ls[j], li[j], v, item);
                            th[j] = ls[j][K - 1];
                        }
                    }
                }
            }
        }
    }

    // ---- merge the two wave halves' lists, write this split's top-k ----
    float* os = a.out_s + static_cast<int64_t>(split) * nq * k;
    int64_t* oi = a.out_i + static_cast<int64_t>(split) * nq * k;
#pragma unroll
    for (int j = 0; j < QS; ++j) {
        // elementwise best of mine[i] vs theirs[K-1-i] is a bitonic sequence
        // holding the top K of the union; a bitonic merge sorts it
        float ms[K];
        uint32_t mi[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const float s2 = __shfl_xor(ls[j][K - 1 - i], 32, 64);
            const uint32_t i2 = static_cast<uint32_t>(__shfl_xor(static_cast<int>(li[j][K - 1 - i]), 32, 64));
            const bool mine = better(ls[j][i], li[j][i], s2, i2);
            ms[i] = mine ? ls[j][i] : s2;
            mi[i] = mine ? li[j][i] : i2;
        }
#pragma unroll
        for (int st = K / 2; st > 0; st >>= 1) {
#pragma unroll
            for (int i = 0; i < K; ++i) {
                if ((i & st) == 0) {
                    const int i2 = i + st;
                    if (better(ms[i2], mi[i2], ms[i], mi[i])) {
                        const float ts = ms[i];
                        const uint32_t ti = mi[i];
                        ms[i] = ms[i2];
                        mi[i] = mi[i2];
                        ms[i2] = ts;
                        mi[i2] = ti;
                    }
                }
            }
        }
        const int64_t q = qb + j * 32 + col;
        if (half == 0 && qok[j]) {
#pragma unroll
            for (int i = 0; i < K; ++i) {
                if (i < k) {
                    const bool ok = mi[i] != kEmptyId;
                    os[q * k + i] = ok ? ms[i] : -FLT_MAX;
                    oi[q * k + i] = ok ? static_cast<int64_t>(mi[i]) + a.id_offset : -1;
                }
            }
        }
    }
}

template <typename T, int S, int K>
int launch_cfg(const Args& a, const Plan& p, hipStream_t st) {
    using C = Cfg<T, S, K>;
    dim3 grid(static_cast<unsigned>((a.nq + C::QT - 1) / C::QT), static_cast<unsigned>(p.splits));
    hipLaunchKernelGGL((flatip_topk_kernel<T, S, K>), grid, dim3(256), 0, st, a, p.items_per_split);
    return check_launch("flatip_topk_kernel");
}

}  // namespace topk
}  // namespace rt

#include "topk_v1.h"
#include "topk_v2.h"
#include "topk_v3.h"
#include "topk_v4.h"
#include "topk_dense.h"

namespace rt {
namespace topk {

// kernel choice: register lists (this file) for fp32 with k <= 32; the
// radix-compacted candidate-buffer kernels for k <= 128 otherwise — topk_v3.h
// for 16-bit d <= 128 with k <= 32 (its scan and threshold refresh win at
// small k), topk_v2.h for the rest (fp32, d > 128, and 32 < k <= 128, where
// v2's buffer schedule measured faster: C4 k=100 4.96 vs 5.15 ms); the sorted
// candidate-buffer kernel (topk_v1.h) above.
// Returns K for the list kernel, 0 for v1, -2 for v2.
inline int list_k(bool f32, int k) {
    if (f32 && k <= 16) return 16;  // small fp32 queries: per-lane register lists (C3, serving)
    if (f32 && k <= 32) return 32;
    return k <= v2::kMaxKv2 ? -2 : 0;
}

// the v2 kernel's LDS image of an fp32 stage exceeds 160 KiB at d > 128: fp32
// d in (128, 256] with k > 32 runs on v1
template <typename T, int S>
constexpr bool v2_fits() { return !(sizeof(T) == 4 && S > 64); }

template <typename T, int S>
int launch_S(const Args& a, const Plan& p, hipStream_t st) {
    constexpr bool F32 = sizeof(T) == 4;
    if constexpr (!F32 && S <= 8) {
        if (p.v4 && p.v4_presample)
            return v4::launch_presampled<T, S, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, p.stride, p.rank,
                                                        a.v4_lists, a.v4_thr, a.fail, st);
        if (p.v4)
            return v4::launch_S<T, S, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, p.stride, p.rank, a.meta,
                                               p.v4_joint ? a.fail : nullptr, st);
    }
    if constexpr (F32) {
        if (p.dense) return dense::launch(a, reinterpret_cast<float*>(a.cand), dense::ld_for(a.nx), st);
        switch (list_k(true, a.k)) {
            case 16: return launch_cfg<T, S, 16>(a, p, st);
            case 32: return launch_cfg<T, S, 32>(a, p, st);
            default: break;
        }
    }
    if constexpr (v2_fits<T, S>()) {
        if (list_k(F32, a.k) == -2) {
            if constexpr (!F32 && S <= 8) {
                if (a.k <= v3::kMaxKv3) return v3::launch_S<T, S>(a, p.splits, p.items_per_split, st);
            }
            return v2::launch_S<T, S>(a, p.splits, p.items_per_split, st);
        }
    }
    return v1::launch_S<T, S>(a, p.cap, p.splits, p.items_per_split, st);
}

// compile-time shape facts the host planner needs, per (dtype, S)
struct Shape {
    int qt, nt, cap;
    int kind;  // 0 register lists, 1 v1, 2 v2
};
template <typename T, int S>
Shape shape_S(int k) {
    switch (list_k(sizeof(T) == 4, k)) {
        case 16: return {Cfg<T, S, 16>::QT, Cfg<T, S, 16>::NT, 0, 0};
        case 32: return {Cfg<T, S, 32>::QT, Cfg<T, S, 32>::NT, 0, 0};
        case -2:
            if (v2_fits<T, S>()) return {v2::kQT, v2::kNT, v2::kCap, 2};
            return {v1::kQT, v1::kNT, v1::cap_for(k), 1};
        default: return {v1::kQT, v1::kNT, v1::cap_for(k), 1};
    }
}

// per-dtype entry points (defined in topk_{f32,f16,bf16}.hip)
int launch_f32(const Args& a, const Plan& p, hipStream_t st);
int launch_f16(const Args& a, const Plan& p, hipStream_t st);
int launch_bf16(const Args& a, const Plan& p, hipStream_t st);
int v4_scan_f16(const Args& a, const Plan& p, int stride, int rank, int mode, hipStream_t st);
int v4_scan_bf16(const Args& a, const Plan& p, int stride, int rank, int mode, hipStream_t st);
Shape shape_f32(int d, int k);
Shape shape_f16(int d, int k);
Shape shape_bf16(int d, int k);

}  // namespace topk
}  // namespace rt
