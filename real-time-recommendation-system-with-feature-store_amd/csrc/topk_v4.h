// Flat-IP top-K for 16-bit corpora (f16 / bf16), d <= 128, k <= 128, on
// large corpora — the C4 shape (65,536 queries x a 125,000-row shard, k = 100)
// and the 1M-row corpus on one GPU. Included by topk_impl.h; replaces
// faiss.IndexFlatIP.search (src/serving/retrieval.py:170-171) on that shape.
//
// Two launches:
//
// 1. flatip_topk_v4_scan: block = 8 waves x QS sets of 32 queries (QS = 2:
//    64 queries per wave, 512 per block; every A fragment read from LDS feeds
//    two MFMAs, and a block's item stream serves 512 queries), over one item
//    split. Rows stream through an LDS ring as in the v3 scan (SADDR
//    LDS-DMA, one pad chunk per row, immediate-offset A fragments): three
//    stages with a barrier inside each, or at d = 128 four stages with a
//    barrier after every other one (see main_pass).
//    Selection runs against a SAMPLED threshold instead of a running one:
//      * sample phase: every `stride`-th stage of the split (a 1/stride
//        sample). Per lane and query set the 16 largest group maxima
//        (group = the 16 rows of a 32-row sub-tile a lane holds) are kept in
//        a sorted register list, one v_med3 per level per insert, no ids.
//      * the estimate: thr = the `rank`-th largest of the query's 32 group
//        maxima (both lane halves). The host picks (stride, rank) so that
//        P(thr > the k-th score) = P(Bin(k, f) >= rank) is below 1e-6 for
//        the sampled fraction f, with rank / f (the expected appends) at
//        most RT_TOPK_V4_APPEND_CAP (topk_api.hip::plan_v4_sample).
//      * main phase: every stage (the sample stages again), each score >= thr
//        appended to the query's candidate buffer (per lane half: one
//        SADDR 8-byte store at the lane's cursor). About rank / f appends
//        per query (~460 at the C4 shapes), against thousands for a running
//        threshold that starts at -inf. A half nearing its capacity is
//        compacted by the v2 radix compaction (threshold raised, never lowered).
//        The filter of a set is a branch-free 16-bit pass mask (two VALU per
//        score, scheduled into the next set's MFMA gaps) and a wave-uniform
//        store loop that runs max-popcount times; the block barrier sits
//        before each stage's last sub-tile so fragments of the next stage are
//        read behind the current MFMAs (see main_pass).
//      * verification: a query whose buffer holds >= k entries (all >= thr)
//        has its split top-k inside it, exactly. A query with fewer (the
//        estimate overshot) makes the whole block rescan the split for its
//        failed queries with thr = -inf and the compaction path of v2 —
//        correct for any data, costly only when it happens.
//      * joint mode (mode 1, several splits): the sample pass covers the
//        whole corpus, so every split of a query derives the same threshold,
//        a lower bound of its corpus-wide k-th; the finish checks the union
//        of the split buffers instead (< k entries: the query is flagged),
//        and a rescue launch pair (mode 2) rebuilds the flagged queries from
//        -inf while every other block exits at once.
//    Each (split, query, half) writes its entry count to `meta`.
// 2. flatip_topk_v4_finish: one wave per query over the union of its split
//    buffers: a radix select on the composite key (order-preserving score
//    key << 32 | ~id, larger = better: score desc, id asc) down to <= 128
//    survivors (usually k plus a few after 16 bits), one 128-entry register
//    bitonic sort, the k best written in Faiss order with (-FLT_MAX, -1)
//    padding.
//    The split merge is part of this pass (no topk_merge launch).
#pragma once

namespace rt {
namespace topk {
namespace v4 {

constexpr int kWavesB = 8;
constexpr int kCap = 1024;             // candidate entries per (split, query)
constexpr int kHalf = kCap / 2;        // per owning lane half
constexpr int kMaxK = 128;
constexpr int kList = 16;              // group maxima per lane and query set (sample phase)
constexpr int kMaxSplits = 16;
constexpr int kSampleList = 32;       // per query: each lane half's 16 largest sampled group maxima, merged
constexpr int kFinishCap = 128;        // survivors a finish wave sorts at once (2 per lane)
constexpr int kFinishRegs = 16;        // candidates per lane the finish holds in registers
#ifndef RT_TOPK_V4_QS
#define RT_TOPK_V4_QS 2
#endif
constexpr int kQS = RT_TOPK_V4_QS;     // query sets of 32 per wave
// one candidate region and cursor per query shared by its two lane halves
// (the lanes (col, 0) and (col, 1) of a query interleave their appends), instead
// of one region per (query, half): half the open buffer lines per block
#ifdef RT_TOPK_V4_PER_HALF
constexpr bool kShared = false;
#else
constexpr bool kShared = true;
#endif

template <int QS>
struct Geo {
    static constexpr int QT = 32 * QS * kWavesB;  // queries per block
};

template <typename T, int S>
struct Cfg4 {
    static_assert(sizeof(T) == 2 && S <= 8, "v4: 16-bit, d <= 128");
    static constexpr int DP = S * 16;
    static constexpr int P = DP * 2 / 16;          // 16-byte data chunks per row
    static constexpr int RS = (P + 1) * 16;        // LDS row stride: one pad chunk
    static constexpr int NT = 128;                 // rows per stage
    static constexpr int NSUB = NT / 32;
    static constexpr int SLOTS = NT * (P + 1);
    static constexpr int PIECES = SLOTS / 64;      // 1 KiB DMA pieces per stage
    static constexpr int MAXP = (PIECES + kWavesB - 1) / kWavesB;
    static constexpr int TILE_BYTES = SLOTS * 16;
#ifdef RT_TOPK_V4_RING3  // A/B: a block barrier inside every stage at d = 128 too
    static constexpr int RING = 3;
#else
    static constexpr int RING = S == 8 ? 4 : 3;    // d = 128: a block barrier every other stage
#endif
    static constexpr int HIST_BYTES = kWavesB * 1024;
    static constexpr int LDS_BYTES = RING * TILE_BYTES + HIST_BYTES + 16;
    static_assert(PIECES * 64 == SLOTS, "whole DMA pieces");
    static_assert(LDS_BYTES <= 163840, "LDS budget");
};

template <int N>
__device__ __forceinline__ void wait_vm_exact() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int LO, int HI>
__device__ __forceinline__ void wait_vm_range(int n) {
    if constexpr (LO == HI) {
        wait_vm_exact<LO>();
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (n <= MID) wait_vm_range<LO, MID>(n);
        else wait_vm_range<MID + 1, HI>(n);
    }
}
// wait until at most n (wave-uniform) vector-memory operations are in flight
__device__ __forceinline__ void wait_vm_le(int n) { wait_vm_range<0, 63>(n < 0 ? 0 : (n > 63 ? 63 : n)); }

// sorted (descending) list insert without ids: l[i] <- med3(l[i], l[i-1], x)
// (= clamp(x, l[i], l[i-1]) since l[i] <= l[i-1]) — one VALU per level
__device__ __forceinline__ void list_insert_med3(float (&l)[kList], float x) {
#pragma unroll
    for (int i = kList - 1; i >= 1; --i) l[i] = __builtin_amdgcn_fmed3f(l[i], l[i - 1], x);
    l[0] = fmaxf(l[0], x);
}

// the union of this lane's list and its partner lane's (lane ^ 32), sorted
// descending into u[0 .. 2 kList)
__device__ __forceinline__ void union_sorted(const float (&l)[kList], float (&u)[2 * kList]) {
#pragma unroll
    for (int i = 0; i < kList; ++i) {
        u[i] = l[i];
        u[2 * kList - 1 - i] = __shfl_xor(l[i], 32, 64);  // partner's list ascending: u is bitonic
    }
#pragma unroll
    for (int st = kList; st > 0; st >>= 1) {
#pragma unroll
        for (int i = 0; i < 2 * kList; ++i) {
            if ((i & st) == 0) {
                const float a = u[i], b = u[i + st];
                u[i] = fmaxf(a, b);
                u[i + st] = fminf(a, b);
            }
        }
    }
}

// the rank-th largest (1-based, rank <= 32) of the union of this lane's list
// and its partner lane's (lane ^ 32); -inf when fewer finite entries exist
__device__ __forceinline__ float union_rank(const float (&l)[kList], int rank) {
    float u[2 * kList];
    union_sorted(l, u);
    float v = -INFINITY;
#pragma unroll
    for (int i = 0; i < 2 * kList; ++i) v = (i == rank - 1) ? u[i] : v;
    return v;
}

// per lane: (bit lane of m) ? b : a, as one v_cndmask_b32
__device__ __forceinline__ float lane_sel(uint64_t m, float a, float b) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// composite key of a candidate: larger = better (score desc, then id asc)
__device__ __forceinline__ uint64_t ckey(const Cand& c) {
    return (static_cast<uint64_t>(v2::okey(c.s)) << 32) | static_cast<uint32_t>(~c.i);
}
__device__ __forceinline__ uint64_t prefix_mask(int shift) { return shift >= 64 ? 0ull : (~0ull << shift); }

// Radix select over candidates visited by each(fn) (whole wave calls; fn gets
// every entry's composite key exactly once, on some lane): 8 bits of the composite key a pass,
// from the top, until the entries whose key's top (64 - shift) bits are >=
// prefix's number <= limit. That set always holds the k best entries (k <=
// limit). Registers: a few; LDS: hist (256 words, this wave's).
template <class Each>
__device__ __forceinline__ void radix_prefix(Each&& each, int k, int limit, uint32_t* hist, uint64_t& prefix,
                                             int& shift, int& kept) {
    const int lane = threadIdx.x & 63;
    int need = k;  // entries still to be found inside the current prefix bucket
    while (shift > 0) {
        // the last pass may have fewer than 8 bits left (the finish starts below
        // the keys' shared prefix, at any bit): its bins are the low 8 bits, the
        // ones above `shift` fixed by the prefix
        const int sh = shift > 8 ? shift - 8 : 0;
        reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_sync();
        const uint64_t pmask = prefix_mask(shift), pre = prefix;
        each([&](uint64_t key) {
            if ((key & pmask) == pre) atomicAdd(&hist[(key >> sh) & 255u], 1u);
        });
        wave_lds_sync();
        const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
        const int c4 = static_cast<int>(h.x + h.y + h.z + h.w);
        int suf = c4;  // inclusive suffix over lanes >= lane (bins ascend with lane)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_down(suf, o, 64);
            if (lane + o < 64) suf += t;
        }
        const int ab = suf - c4;
        const int c3 = ab + static_cast<int>(h.w), c2 = c3 + static_cast<int>(h.z);
        const int c1 = c2 + static_cast<int>(h.y), c0 = c1 + static_cast<int>(h.x);
        const bool hit = ab < need && c0 >= need;
        const uint64_t bm = __ballot(hit);
        const int src = bm ? __builtin_ctzll(bm) : 0;
        const int bl = c3 >= need ? 3 : c2 >= need ? 2 : c1 >= need ? 1 : 0;
        const int al = c3 >= need ? ab : c2 >= need ? c3 : c1 >= need ? c2 : c1;
        const int inb = c3 >= need   ? static_cast<int>(h.w)
                        : c2 >= need ? static_cast<int>(h.z)
                        : c1 >= need ? static_cast<int>(h.y)
                                     : static_cast<int>(h.x);
        const int bin = __shfl(4 * lane + bl, src, 64);
        const int above = __shfl(al, src, 64);
        const int inbin = __shfl(inb, src, 64);
        wave_lds_sync();
        prefix |= static_cast<uint64_t>(bin) << sh;
        shift = sh;
        need -= above;
        kept = (k - need) + inbin;  // strictly above the bucket + the bucket
        if (kept <= limit) break;
    }
}

// In-scan compaction of one query's buffer (halves of n0 / n1 entries, k <=
// n0 + n1), streamed from memory so that the scan keeps its registers: each
// half keeps, in place and in order, its entries in the radix bucket holding
// the k best (<= limit entries in all). thr = the new filter threshold:
// the bucket's score floor (v >= thr), or, when the bucket had to be resolved
// down into the ids (massive exact ties), strictly above the k-th score — items
// arrive in increasing id order, so an equal later score loses.
__device__ __forceinline__ void compact_stream(Cand* __restrict__ buf, int& n0, int& n1, int k, int limit,
                                               uint32_t* hist, float& thr) {
    const int lane = threadIdx.x & 63;
    __threadfence_block();
    const int a0 = n0, a1 = n1;
    auto each = [&](auto&& fn) {
        for (int i = lane; i < a0; i += 64) fn(ckey(buf[i]));
        for (int i = lane; i < a1; i += 64) fn(ckey(buf[kHalf + i]));
    };
    uint64_t prefix = 0;
    int shift = 64, kept = a0 + a1;
    radix_prefix(each, k, limit, hist, prefix, shift, kept);
    const uint64_t pmask = prefix_mask(shift);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Cand* p = buf + h * kHalf;
        const int n = h ? a1 : a0;
        int m = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            Cand c{-INFINITY, kEmptyId};
            bool take = false;
            if (i < n) {
                c = p[i];
                take = (ckey(c) & pmask) >= prefix;
            }
            const uint64_t bm = __ballot(take);
            const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                    static_cast<uint32_t>(bm >> 32),
                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
            if (take) p[pos] = c;  // pos <= i: every lane read its entry before any lane writes
            m += __popcll(bm);
        }
        if (h) n1 = m;
        else n0 = m;
    }
    const float floor = v2::okey_inv(static_cast<uint32_t>(prefix >> 32));
    if (shift >= 32) thr = (static_cast<uint32_t>(prefix >> 32) <= 0x007FFFFFu) ? -FLT_MAX : floor;
    else thr = nextafterf(floor, INFINITY);
    __threadfence_block();
}

template <typename T, int S, int QS, bool EXCL>
__global__ __launch_bounds__(512) void flatip_topk_v4_scan(Args a, int splits, int64_t items_per_split, int stride,
                                                            int rank, int* __restrict__ meta, int mode,
                                                            const int* __restrict__ fail) {
    using M = Mfma<T>;
    using C = Cfg4<T, S>;
    typedef typename M::frag frag;
    constexpr int QT = Geo<QS>::QT;
    __shared__ __attribute__((aligned(1024))) char lds[C::LDS_BYTES];
    char* const ring = lds;
    uint32_t* const hist_all = reinterpret_cast<uint32_t*>(lds + C::RING * C::TILE_BYTES);
    uint32_t* const flag = hist_all + kWavesB * 256;

    const T* __restrict__ Q = reinterpret_cast<const T*>(a.Q);
    const char* __restrict__ Xb = reinterpret_cast<const char*>(a.X);
    const int d = a.d, k = a.k;
    const int64_t nq = a.nq;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    const int split = static_cast<int>(blockIdx.x % static_cast<unsigned>(splits));
    const int64_t qtile = blockIdx.x / static_cast<unsigned>(splits);
    const int64_t qw = qtile * QT + wave * (32 * QS);  // wave's first query
    const int64_t i_begin = static_cast<int64_t>(split) * items_per_split;
    const int64_t i_end = (i_begin + items_per_split) < a.nx ? (i_begin + items_per_split) : a.nx;
    const int64_t row_bytes = static_cast<int64_t>(d) * 2;
    const int64_t q_pad = static_cast<int64_t>(gridDim.x / splits) * QT;
    Cand* const cbase = a.cand + (static_cast<int64_t>(split) * q_pad + qw) * kCap;  // wave's 32·QS buffers
    uint32_t* const whist = hist_all + wave * 256;
    const int nst = i_end > i_begin ? static_cast<int>((i_end - i_begin + C::NT - 1) / C::NT) : 0;
    // mode 0: per-split sample, per-split verification (rescan on failure);
    // mode 1 (joint): the sample pass covers the WHOLE corpus, so every split of
    //   a query derives the same threshold, a lower bound of the query's k-th
    //   over the corpus; no per-split verification (the finish checks the union);
    // mode 2 (rescue): only queries the finish flagged (union < k) run, from -inf.
    // mode 3 (presample): the sample pass over this block's own split only, per
    //   query the union of each lane half's 16 largest group maxima (a subset
    //   of the split's 32 largest: a threshold from it can only be lower, i.e.
    //   safe) to a.lists_out; no main pass
    //   (flatip_topk_v4_threshold turns the lists of all splits — or of all
    //   ranks' shards — into one threshold per query);
    // mode 4: no sample pass, thr = a.thr_in[query], then the main pass.
    const bool joint = mode == 1;
    // rows [p_begin, p_end) of the current pass (fetch, tail masks, stages)
    int64_t p_begin = joint ? 0 : i_begin, p_end = joint ? a.nx : i_end;
    const int nst_s = joint ? static_cast<int>((a.nx + C::NT - 1) / C::NT) : nst;
    const int nsa = (mode != 2 && mode != 4 && rank > 0 && stride > 0) ? (nst_s + stride - 1) / stride : 0;  // sample stages
    if (tid == 0) *flag = 0u;
    if (mode == 2) {  // rescue: exit before any load unless a query of this block was flagged
        __syncthreads();  // *flag zeroed above
        bool any = false;
#pragma unroll
        for (int j = 0; j < QS; ++j) {
            const int64_t q = qw + j * 32 + col;
            any |= q < nq && fail[q] != 0;
        }
        if (__ballot(any) != 0 && lane == 0) atomicOr(flag, 1u);
        __syncthreads();
        if (*flag == 0u) return;  // block-uniform (the common case: nothing flagged)
        __syncthreads();          // every wave has read the flag before it is reused below
        if (tid == 0) *flag = 0u;
    }

    frag qf[QS][S];
    bool qok[QS];
    const uint32_t* excl[QS];
#pragma unroll
    for (int j = 0; j < QS; ++j) {
        const int64_t q = qw + j * 32 + col;
        qok[j] = q < nq;
        const T* qrow = Q + (qok[j] ? q : 0) * d;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k0 = 16 * s + 8 * half;
            if (qok[j] && k0 < d) qf[j][s] = frag_from<T>(qrow + k0);
            else qf[j][s] = frag{};
        }
        excl[j] = (EXCL && qok[j]) ? a.excl + q * a.excl_words : nullptr;
    }
#pragma unroll
    for (int j = 0; j < QS; ++j)
#pragma unroll
        for (int s = 0; s < S; ++s) {  // drained here, not at the loop header's merged wait
            const uint4 t = __builtin_bit_cast(uint4, qf[j][s]);
            asm volatile("" ::"v"(t.x), "v"(t.y), "v"(t.z), "v"(t.w));
        }

    // ---- append cursors: byte offset of the lane's next entry from the wave's base ----
    const uint32_t wb_lo = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase))));
    const uint32_t wb_hi = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase) >> 32)));
    const uint64_t wbase = (static_cast<uint64_t>(wb_hi) << 32) | wb_lo;
    // wave-uniform global base: the appends compile to SADDR global stores
    // (a generic pointer would give flat stores, counted in lgkmcnt too)
    __attribute__((address_space(1))) char* const wbytes =
        reinterpret_cast<__attribute__((address_space(1))) char*>(wbase);
    uint32_t woff0[QS], woff[QS];
    float thr[QS];
#pragma unroll
    for (int j = 0; j < QS; ++j) {
        woff0[j] = static_cast<uint32_t>(((j * 32 + col) * kCap + (kShared ? 0 : half * kHalf)) * sizeof(Cand));
        woff[j] = woff0[j];
        thr[j] = qok[j] ? -FLT_MAX : INFINITY;
    }
    if (mode == 2) {  // rescue: the flagged queries from -inf (a running threshold), the rest skip
#pragma unroll
        for (int j = 0; j < QS; ++j) thr[j] = (qok[j] && fail[qw + j * 32 + col] != 0) ? -FLT_MAX : INFINITY;
    }
    if (mode == 4) {  // external per-query thresholds (a presample over every split / every shard)
#pragma unroll
        for (int j = 0; j < QS; ++j) thr[j] = qok[j] ? fmaxf(a.thr_in[qw + j * 32 + col], -FLT_MAX) : INFINITY;
    }
    constexpr int kHead = C::NSUB * 16;  // appends per half between two compaction checks, at most
    // shared region: both halves append up to kHead each between checks
    constexpr int kRoom = kShared ? kCap - 2 * kHead : kHalf - kHead;
    constexpr uint32_t kLimBytes = static_cast<uint32_t>(kRoom * sizeof(Cand));
    constexpr int kLimit = kRoom;  // a compaction keeps at most this many entries (in all)

    // ---- DMA plan (as v3): this wave's pieces w, w+8, ... of a stage ----
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int npieces = (C::PIECES - wave_u + kWavesB - 1) / kWavesB;
    const int row_vecs = d / 8;
    uint32_t soff[C::MAXP];
#pragma unroll
    for (int i = 0; i < C::MAXP; ++i) {
        const int o = (wave_u + kWavesB * i) * 64 + lane;
        const int r = o / (C::P + 1), c = o % (C::P + 1);
        soff[i] = static_cast<uint32_t>(r * static_cast<int>(row_bytes) + (c < row_vecs ? c * 16 : 0));
    }
    const uint32_t ring0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) char*)(ring)));
    int issued = 0;
    int mk[C::RING - 1];
    auto fetch = [&](int64_t t0, int buf) {
        const uint32_t base = ring0 + buf * C::TILE_BYTES + wave_u * 1024;
        const uint64_t sbu = reinterpret_cast<uint64_t>(Xb + t0 * row_bytes);
        const int rem = static_cast<int>(p_end - t0 < C::NT ? p_end - t0 : C::NT);
#pragma unroll
        for (int i = 0; i < C::MAXP; ++i) {
            if (i < npieces) {
                uint32_t off = soff[i];
                if (rem < C::NT) {  // rows past the split end read its last row (masked)
                    const int r = ((wave_u + kWavesB * i) * 64 + lane) / (C::P + 1);
                    if (r >= rem) off -= static_cast<uint32_t>((r - (rem - 1)) * row_bytes);
                }
                unsigned keep;
                // s_nop 4: the SGPR operands may come straight from a VALU (a spill
                // reload), which a VMEM read as base needs 5 wait states after
                asm volatile(
                    "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                    "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(off), "s"(sbu), "s"(base + i * (kWavesB * 1024))
                    : "memory");
            }
        }
        issued += npieces;
    };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // ---- selection (per query set j) ----
    auto max16 = [&](const f32x16& acc) {
        float m = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, acc[r]), acc[r + 1]);
        return fmaxf(m, acc[15]);
    };
    // Appends of one sub-tile for query set j, in two parts so that the
    // compares never wait on a branch:
    //  * passmask: the 16 compares fold into a per-lane 16-bit mask (bit r =
    //    row (r & 3) + 8 (r >> 2) of the lane's half passes) with no branch;
    //    the caller schedules them into the gaps of the next set's MFMAs.
    //  * store_loop: a wave-uniform loop that runs max-popcount times (0 or 1
    //    on almost every sub-tile), each lane storing its lowest passing row
    //    (the score picked by a 4-level select on that row's bits) with one
    //    SADDR dwordx2 store at its cursor.
    // Rows ascend with r, so each lane appends the same entries in the same
    // order as a row-by-row filter would.
    auto passmask = [&](int j, const f32x16& acc, int64_t sub0, uint32_t tm) -> uint32_t {
        const float t = thr[j];
        uint32_t pm = 0u;
        // pm = 2 pm + (acc[r] >= t), rows 15..0: two VALU per row, no wait
        // states (written in C the compiler emits compare, cndmask and or/shift,
        // with an s_nop between the compare and the cndmask that reads vcc)
#pragma unroll
        for (int r = 15; r >= 0; --r)
            asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                : "+v"(pm)
                : "v"(acc[r]), "v"(t)
                : "vcc");
        pm &= tm;
        if constexpr (EXCL) {
            if (excl[j]) {
                const uint32_t xw = excl[j][sub0 >> 5];  // sub0 is 32-aligned: one bitmap word per sub-tile
                // this half's rows 4h + {0..3, 8..11, 16..19, 24..27} -> bits r = 0..15
                const uint32_t xh = xw >> (4 * half);
                const uint32_t xr = (xh & 0xFu) | ((xh >> 4) & 0xF0u) | ((xh >> 8) & 0xF00u) | ((xh >> 12) & 0xF000u);
                pm &= ~xr;
            }
        }
        return pm;
    };
#ifdef RT_TOPK_V4_STREAMTEST
    uint32_t scur = 0u;
#endif
    auto store_loop = [&](int j, uint32_t pm, const f32x16& acc, int64_t sub0) {
        const uint32_t sub_lane = static_cast<uint32_t>(sub0) + static_cast<uint32_t>(4 * half);
        uint32_t wo = woff[j];
        while (true) {
            const uint64_t sb = __ballot(pm != 0u);
            if (sb == 0ull) break;
            issued += 1;  // exactly one store instruction (dwordx2) for the wave
            // shared region: the half-1 lane writes behind its half-0 partner
            // when both store this round; both advance by the pair's stores
            uint32_t other = 0u, slot = wo;
            if constexpr (kShared) {
                other = static_cast<uint32_t>((sb >> (lane ^ 32)) & 1ull);
                slot = wo + (half ? other * static_cast<uint32_t>(sizeof(Cand)) : 0u);
            }
#ifdef RT_TOPK_V4_STREAMTEST  // timing probe only: wave-contiguous appends (the finish reads garbage)
            slot = ((scur + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(sb >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(sb), 0u))) &
                    (64u * kCap - 1u)) * static_cast<uint32_t>(sizeof(Cand));
            scur += static_cast<uint32_t>(__popcll(sb));
#endif
            if (pm) {
                // the lowest passing row as an isolated bit, tested against
                // constant masks; the score is picked by explicit v_cndmask
                // instructions (written as selects on acc[], the compiler folds
                // them into a 16-way variable-index extract of the vector)
                const uint32_t lb = pm & (0u - pm);
                pm ^= lb;
                const bool b0 = (lb & 0xAAAAu) != 0u, b1 = (lb & 0xCCCCu) != 0u;
                const bool b2 = (lb & 0xF0F0u) != 0u, b3 = (lb & 0xFF00u) != 0u;
                const uint64_t m0 = __ballot(b0), m1 = __ballot(b1), m2 = __ballot(b2), m3 = __ballot(b3);
                float v8[8], v4[4], v2[2];
#pragma unroll
                for (int i = 0; i < 8; ++i) v8[i] = lane_sel(m0, acc[2 * i], acc[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 4; ++i) v4[i] = lane_sel(m1, v8[2 * i], v8[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 2; ++i) v2[i] = lane_sel(m2, v4[2 * i], v4[2 * i + 1]);
                const float s = lane_sel(m3, v2[0], v2[1]);
                const uint32_t id = sub_lane + (b0 ? 1u : 0u) + (b1 ? 2u : 0u) + (b2 ? 8u : 0u) + (b3 ? 16u : 0u);
                // a compiler-visible SADDR store (hipcc counts it and pads its hazards)
                *reinterpret_cast<__attribute__((address_space(1))) uint64_t*>(wbytes + slot) =
                    (static_cast<uint64_t>(id) << 32) | __float_as_uint(s);
                if constexpr (!kShared) wo += 8;
            }
            if constexpr (kShared)
                wo += static_cast<uint32_t>(sizeof(Cand)) * (((sb >> lane) & 1ull ? 1u : 0u) + other);
        }
        woff[j] = wo;
    };
    // rows of a sub-tile with `left` (< 32) valid rows, as this lane's pass-mask bits
    auto tail_bits = [&](int left) -> uint32_t {
        const int lim = left - 4 * half;
        uint32_t m = 0u;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            int c = lim - 8 * g;
            c = c < 0 ? 0 : (c > 4 ? 4 : c);
            m |= ((1u << c) - 1u) << (4 * g);
        }
        return m;
    };
    // compact every buffer of this wave that may overflow before the next check
    auto maybe_compact = [&]() {
#pragma unroll
        for (int j = 0; j < QS; ++j) {
            const uint64_t m = __ballot(woff[j] - woff0[j] > kLimBytes);
            uint32_t need = static_cast<uint32_t>(m) | static_cast<uint32_t>(m >> 32);
            if (!need) continue;
            while (need) {
                const int c = __builtin_ctz(need);
                need &= need - 1;
                const int cnt = static_cast<int>((woff[j] - woff0[j]) / sizeof(Cand));
                int n0 = __shfl(cnt, c, 64), n1 = kShared ? 0 : __shfl(cnt, c + 32, 64);
                float nt;
                compact_stream(cbase + static_cast<int64_t>(j * 32 + c) * kCap, n0, n1, k, kLimit, whist, nt);
                if (col == c) {
                    woff[j] = woff0[j] + static_cast<uint32_t>(((half && !kShared) ? n1 : n0) * sizeof(Cand));
                    thr[j] = fmaxf(thr[j], nt);
                }
            }
#pragma unroll
            for (int i = 0; i < C::RING - 1; ++i) mk[i] = issued;  // drained
        }
    };

    // ---- MFMA sub-tiles ----
    const int a_lane = col * C::RS + half * 16;
    auto lds_a = [&](frag (&af)[S], const char* stage, int rt) {
#pragma unroll
        for (int s = 0; s < S; ++s)
            af[s] = __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(stage + rt * 32 * C::RS + s * 32));
    };
    auto mask_tail = [&](f32x16& acc, int64_t sub0) {
        const int left = static_cast<int>(p_end - sub0);
        if (left < 32) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (tile_row(r, half) >= left) acc[r] = -INFINITY;
        }
    };
    auto mask_excl = [&](int j, f32x16& acc, int64_t sub0) {
        if constexpr (EXCL) {
            if (excl[j]) {
                const uint32_t xw = excl[j][sub0 >> 5];
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if ((xw >> tile_row(r, half)) & 1u) acc[r] = -INFINITY;
            }
        }
    };

    // stage v of a pass: rows [stage_row(v), +NT); `sample` passes visit every
    // stride-th stage
    auto stage_t0 = [&](int v, bool sample) -> int64_t {
        return p_begin + static_cast<int64_t>(sample ? v * stride : v) * C::NT;
    };

    // ---- sample pass: group-max lists ----
    float L[QS][kList];
#pragma unroll
    for (int j = 0; j < QS; ++j)
#pragma unroll
        for (int i = 0; i < kList; ++i) L[j][i] = -INFINITY;

    auto prologue = [&](int nv, bool sample) {
        int mark0 = 0;
#pragma unroll
        for (int b = 0; b < C::RING - 1; ++b) {
            if (b < nv) fetch(stage_t0(b, sample), b);
            if (b == 0) mark0 = issued;
            else mk[b - 1] = issued;
        }
        wait_vm_le(issued - mark0);
        raw_barrier();
    };

    RT_PT(uint64_t pc_wait = 0, pc_bar = 0, pc_main = 0, pc_samp = 0, pc_cmp = 0; const uint64_t pc_start = clock64();)
    if (nsa > 0) {
        prologue(nsa, true);
        int cur = 0;
        for (int v = 0; v < nsa; ++v) {
            const int64_t t0 = stage_t0(v, true);
            const bool more = v + 1 < nsa;
            const int rem = static_cast<int>(p_end - t0 < C::NT ? p_end - t0 : C::NT);
            if (v + C::RING - 1 < nsa) fetch(stage_t0(v + C::RING - 1, true), cur == 0 ? C::RING - 1 : cur - 1);
            mk[C::RING - 2] = issued;
            const char* stage = ring + cur * C::TILE_BYTES + a_lane;
#pragma unroll
            for (int rt = 0; rt < C::NSUB; ++rt) {
                if (rt * 32 < rem) {
                    frag af[S];
                    lds_a(af, stage, rt);
                    f32x16 acc[QS];
#pragma unroll
                    for (int j = 0; j < QS; ++j) {
                        acc[j] = f32x16{};
#pragma unroll
                        for (int s = 0; s < S; ++s) acc[j] = M::run(af[s], qf[j][s], acc[j]);
                    }
                    const int64_t sub0 = t0 + rt * 32;
#pragma unroll
                    for (int j = 0; j < QS; ++j) {
                        if (rem < (rt + 1) * 32) mask_tail(acc[j], sub0);
                        mask_excl(j, acc[j], sub0);
                        list_insert_med3(L[j], max16(acc[j]));
                    }
                }
            }
            if (more) wait_vm_le(issued - mk[0]);
            raw_barrier();
#pragma unroll
            for (int i = 0; i + 1 < C::RING - 1; ++i) mk[i] = mk[i + 1];
            cur = cur == C::RING - 1 ? 0 : cur + 1;
        }
        RT_PT(pc_samp = clock64() - pc_start;)
        if (mode == 3) {  // presample: both lane halves' 16 largest group maxima per query, merged and sorted
#pragma unroll
            for (int j = 0; j < QS; ++j) {
                float u[2 * kList];
                union_sorted(L[j], u);
                if (half == 0 && qok[j]) {
                    float4* o = reinterpret_cast<float4*>(
                        a.lists_out + ((static_cast<int64_t>(split) * q_pad) + qw + j * 32 + col) * kSampleList);
#pragma unroll
                    for (int i = 0; i < kSampleList / 4; ++i)
                        o[i] = make_float4(u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3]);
                }
            }
            return;  // block-uniform: mode 3 runs no main pass
        }
#pragma unroll
        for (int j = 0; j < QS; ++j) {
            const float e = union_rank(L[j], rank);
            if (qok[j]) thr[j] = e > -FLT_MAX ? e : -FLT_MAX;
        }
    }
    if (mode == 3) {  // an empty split (no sample stages): no candidates to report
#pragma unroll
        for (int j = 0; j < QS; ++j)
            if (half == 0 && qok[j]) {
                float4* o = reinterpret_cast<float4*>(
                    a.lists_out + ((static_cast<int64_t>(split) * q_pad) + qw + j * 32 + col) * kSampleList);
#pragma unroll
                for (int i = 0; i < kSampleList / 4; ++i) o[i] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
            }
        return;
    }
    p_begin = i_begin;  // the main pass covers this block's split
    p_end = i_end;

    // ---- main pass over every stage ----
    // * A fragments of sub-tile t+1 are read behind the MFMAs of t's last set
    //   (across a stage boundary too), so no LDS read latency is exposed.
    // * set QS-1 of sub-tile t is filtered behind set 0's MFMAs of t+1.
    // * the block barrier sits BEFORE a stage's last sub-tile, not between
    //   stages: there every wave has waited for its own DMA pieces of stage
    //   v+1 (so after the barrier stage v+1 is visible and the last sub-tile
    //   can already read its fragments), and every wave is past stage v-1, so
    //   stage v+2 is DMA'd into that buffer right after it. The DMA has one
    //   stage to land.
    // RING = 4 (d = 128; 4 x 34.8 KB ring): the block barrier sits at the END of every
    // odd stage v instead of inside every stage. Before it each wave waits for
    // its pieces of stages v+1 and v+2 (DMA'd two stages earlier); after it,
    // stages v+3 and v+4 go into the buffers of v-1 and v, and stage v+1's first
    // fragments are re-read (the prefetch in v's last sub-tile may have read
    // them before they landed). Waves drift apart by up to two stages between
    // barriers instead of one sub-tile.
    constexpr bool R4 = C::RING == 4;
    auto main_pass = [&]() {
        if (nst == 0) return;
        int mk_next;
        if constexpr (R4) {
            fetch(stage_t0(0, false), 0);
            if (nst > 1) fetch(stage_t0(1, false), 1);
            const int m01 = issued;
            if (nst > 2) fetch(stage_t0(2, false), 2);
            if (nst > 3) fetch(stage_t0(3, false), 3);
            mk_next = issued;
            wait_vm_le(issued - m01);
            raw_barrier();
        } else {
            fetch(stage_t0(0, false), 0);
            const int mark0 = issued;
            if (nst > 1) fetch(stage_t0(1, false), 1);
            mk_next = issued;
            wait_vm_le(issued - mark0);
            raw_barrier();
        }
        frag af[S];
        f32x16 acc[QS];
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[QS - 1][r] = -INFINITY;  // "previous" of the first sub-tile
        f32x16 accp = acc[QS - 1];                                 // (QS = 1: the previous sub-tile)
        int64_t sub_prev = i_begin;
        uint32_t tm_prev = 0u;  // no rows: the first sub-tile has no previous set
        int cur = 0;
        lds_a(af, ring + a_lane, 0);
        // pins a set's MFMAs above the store loop that follows them (without it the
        // compiler sinks the MFMAs below the loop, into the block that reads them)
        auto pin = [&](f32x16& x) { asm volatile("" : "+v"(x)); };
        // MFMA s of a set, then (optionally) the next sub-tile's fragment s and
        // 5 VALU (the previous set's compares)
        auto interleave = [&](bool with_reads, bool with_valu) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (with_reads) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (with_valu) __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            }
        };
        for (int v = 0; v < nst; ++v) {
            const int64_t t0 = stage_t0(v, false);
            const bool more = v + 1 < nst;
            const int rem = static_cast<int>(i_end - t0 < C::NT ? i_end - t0 : C::NT);
            const char* stage = ring + cur * C::TILE_BYTES + a_lane;
            const char* nstage = ring + (cur == C::RING - 1 ? 0 : cur + 1) * C::TILE_BYTES + a_lane;
            RT_PT(uint64_t c0 = clock64();)
#pragma unroll
            for (int rt = 0; rt < C::NSUB; ++rt) {
                if (!R4 && rt == C::NSUB - 1) {
                    RT_PT(const uint64_t c1 = clock64(); pc_main += c1 - c0;)
                    if (more) wait_vm_le(issued - mk_next);
                    RT_PT(const uint64_t c2 = clock64(); pc_wait += c2 - c1;)
                    raw_barrier();
                    RT_PT(const uint64_t c3 = clock64(); pc_bar += c3 - c2;)
                    if (more) {
                        maybe_compact();  // fragments of this sub-tile are live (in registers)
                        if (v + 2 < nst) fetch(stage_t0(v + 2, false), cur == 0 ? C::RING - 1 : cur - 1);
                        mk_next = issued;
                    }
                    RT_PT(c0 = clock64(); pc_cmp += c0 - c3;)
                }
                if (rt * 32 < rem) {
                    const int64_t sub0 = t0 + rt * 32;
                    // the next sub-tile's rows: this stage, or the next stage's first
                    // (rows past a partial stage's end are stale but finite, never filtered in)
                    // (always a valid LDS address: after the last stage the reads are unused)
                    constexpr bool nxt = true;
                    const char* nsrc = rt + 1 < C::NSUB ? stage + (rt + 1) * 32 * C::RS : nstage;
                    uint32_t tm = 0xFFFFu;  // rows past a partial stage's end: masked here
                    if (rem < (rt + 1) * 32) tm = tail_bits(rem - rt * 32);
                    // set 0: MFMAs, with the previous sub-tile's last set compared in their gaps
                    acc[0] = f32x16{};
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        acc[0] = M::run(af[s], qf[0][s], acc[0]);
                        if (QS == 1 && nxt)
                            af[s] = __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(nsrc + s * 32));
                    }
                    if constexpr (QS > 1) {
                        const uint32_t pm = passmask(QS - 1, acc[QS - 1], sub_prev, tm_prev);
                        interleave(false, true);
                        pin(acc[0]);
                        store_loop(QS - 1, pm, acc[QS - 1], sub_prev);
                    } else {  // one set: the previous sub-tile's scores wait in accp
                        const uint32_t pm = passmask(0, accp, sub_prev, tm_prev);
                        interleave(nxt, true);
                        pin(acc[0]);
                        store_loop(0, pm, accp, sub_prev);
                        accp = acc[0];
                    }
#pragma unroll
                    for (int j = 1; j < QS; ++j) {
                        acc[j] = f32x16{};
#pragma unroll
                        for (int s = 0; s < S; ++s) {
                            acc[j] = M::run(af[s], qf[j][s], acc[j]);
                            // fragment s is free once its last MFMA issued
                            if (j == QS - 1 && nxt)
                                af[s] = __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(nsrc + s * 32));
                        }
                        const uint32_t pm = passmask(j - 1, acc[j - 1], sub0, tm);
                        interleave(j == QS - 1 && nxt, true);
                        pin(acc[j]);
                        store_loop(j - 1, pm, acc[j - 1], sub0);
                    }
                    sub_prev = sub0;
                    tm_prev = tm;
                }
            }
            RT_PT(pc_main += clock64() - c0;)
            if constexpr (R4) {
                if (more) maybe_compact();  // wave-local: one stage of appends between checks
                if (more && (v & 1)) {
                    wait_vm_le(issued - mk_next);  // this wave's pieces of stages v+1, v+2
                    raw_barrier();
                    if (v + 3 < nst) fetch(stage_t0(v + 3, false), (v + 3) & 3);
                    if (v + 4 < nst) fetch(stage_t0(v + 4, false), v & 3);
                    mk_next = issued;
                    lds_a(af, nstage, 0);
                }
            }
            cur = cur == C::RING - 1 ? 0 : cur + 1;
        }
        if constexpr (QS > 1) store_loop(QS - 1, passmask(QS - 1, acc[QS - 1], sub_prev, tm_prev), acc[QS - 1], sub_prev);
        else store_loop(0, passmask(0, accp, sub_prev, tm_prev), accp, sub_prev);
        maybe_compact();
    };
#ifdef RT_TOPK_PROBE_NOSEL
#pragma unroll
    for (int j = 0; j < QS; ++j) thr[j] = INFINITY;  // probe builds only: the scan without appends
#endif
    main_pass();

    // ---- verification: a sampled threshold that left < k entries rescans ----
#ifdef RT_TOPK_PROBE_NOSEL
    if (false) {
#else
    if (mode == 0 && nsa > 0) {
#endif
        bool any = false;
#pragma unroll
        for (int j = 0; j < QS; ++j) {
            const int cnt = static_cast<int>((woff[j] - woff0[j]) / sizeof(Cand));
            const int tot = kShared ? cnt : cnt + __shfl_xor(cnt, 32, 64);
            const bool fail = qok[j] && tot < k;
            any |= fail;
            if (fail) {
                thr[j] = -FLT_MAX;  // start over for this query: empty buffer, v2 selection
                woff[j] = woff0[j];
            } else {
                thr[j] = INFINITY;  // done: no appends in the rescan
            }
        }
        if (__ballot(any) != 0 && lane == 0) atomicOr(flag, 1u);
        __syncthreads();
        if (*flag) main_pass();  // block-uniform
    }

    // ---- entry counts for the finish pass ----
#pragma unroll
    for (int j = 0; j < QS; ++j) {
        const int cnt = static_cast<int>((woff[j] - woff0[j]) / sizeof(Cand));
        // shared region: the whole count in the half-0 segment, the half-1 segment empty
        meta[((static_cast<int64_t>(split) * q_pad) + qw + j * 32 + col) * 2 + half] = (kShared && half) ? 0 : cnt;
    }
#ifdef RT_TOPK_PROBE_TIMING
    {  // [total, DMA wait, barrier, main sub-tiles, sample pass, compaction checks]
        const int64_t gw = static_cast<int64_t>(blockIdx.x) * kWavesB + wave;
        if (lane == 0 && gw < 65536) {
            uint64_t* o = v3::probe_cycles + gw * 6;
            o[0] = clock64() - pc_start; o[1] = pc_wait; o[2] = pc_bar; o[3] = pc_main; o[4] = pc_samp; o[5] = pc_cmp;
        }
    }
#endif
}

// ---- finish: radix select over the union of a query's split buffers ----

template <int E>
__device__ __noinline__ void finish_sort(const Cand* __restrict__ buf, int m, int k, float* __restrict__ os,
                                         int64_t* __restrict__ oi, int64_t id_offset) {
    const int lane = threadIdx.x & 63;
    float s[E];
    uint32_t id[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int r = lane * E + j;
        const Cand c = r < m ? buf[r] : Cand{-INFINITY, kEmptyId};
        s[j] = c.s;
        id[j] = c.i;
    }
#ifndef RT_SORT2_GENERIC  // A/B: the loop form
    if constexpr (E == 2) wave_sort_regs2(s, id);
    else
#endif
        wave_sort_regs<E>(s, id);
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int r = lane * E + j;
        if (r < k) {
            const bool ok = id[j] != kEmptyId;
            os[r] = ok ? s[j] : -FLT_MAX;
            oi[r] = ok ? static_cast<int64_t>(id[j]) + id_offset : -1;
        }
    }
}

// one wave per query; block = 4 waves (a template only so that the three
// per-dtype translation units that include this header share one definition)
template <int NW = 4>
__global__ __launch_bounds__(256) void flatip_topk_v4_finish(const Cand* __restrict__ cand,
                                                             const int* __restrict__ meta, int splits,
                                                             int64_t q_pad, int64_t nq, int k,
                                                             float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                             int64_t id_offset, int mode, int* __restrict__ fail) {
    __shared__ __attribute__((aligned(16))) uint32_t hist_all[4][256];
    __shared__ __attribute__((aligned(16))) Cand keep_all[4][kFinishCap];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (q >= nq) return;
    if (mode == 2 && fail[q] == 0) return;
    uint32_t* hist = hist_all[w];
    Cand* keep = keep_all[w];
    const int nseg = 2 * splits;
    // segment (split s, half h) = lane 2s+h: entry count and exclusive prefix
    int cnt = 0;
    if (lane < nseg) cnt = meta[((static_cast<int64_t>(lane >> 1) * q_pad) + q) * 2 + (lane & 1)];
    int pre = cnt;  // inclusive prefix over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(pre, o, 64);
        if (lane >= o) pre += t;
    }
    const int total = __shfl(pre, 63, 64);
    // mode 1 (joint threshold): the union of the split buffers must hold k
    // entries, else the query is flagged for the rescue pair of launches;
    // mode 2: only the flagged queries (their buffers rebuilt from -inf)
    if (mode == 1) {
        const bool short_ = total < k;
        if (lane == 0) fail[q] = short_ ? 1 : 0;
        if (short_) return;
    }
    auto seg_ptr = [&](int sg) {
        return cand + ((static_cast<int64_t>(sg >> 1) * q_pad) + q) * kCap + (sg & 1) * kHalf;
    };
    // visit every entry: fn(entry); segments in order, lanes strided
    auto each = [&](auto&& fn) {
        for (int sg = 0; sg < nseg; ++sg) {
            const int n = __shfl(cnt, sg, 64);
            const Cand* p = seg_ptr(sg);
            for (int i = lane; i < n; i += 64) fn(ckey(p[i]));
        }
    };
    float* os = out_s + q * k;
    int64_t* oi = out_i + q * k;

    if (total <= 64 * kFinishRegs) {
        // Register path (the C4 shapes: ~700 candidates): every candidate is
        // read ONCE, as its composite key, into this lane's slots f = e*64 + lane
        // of the segments' concatenation. The radix select then starts below
        // the bits all keys share (scores above one threshold agree in sign,
        // exponent and the top mantissa bits), so its first pass already
        // splits them, and no pass re-reads memory.
        int bnd[2 * kMaxSplits];  // inclusive segment ends (wave-uniform)
#pragma unroll
        for (int t = 0; t < 2 * kMaxSplits; ++t) bnd[t] = __builtin_amdgcn_readlane(pre, t);
        uint64_t key[kFinishRegs];
        uint64_t mx = 0ull, mn = ~0ull;
        // all loads issued before any is used; the segment of slot f found by
        // a search over NS - 1 boundaries (NS = 4: the 2-split C4 plans)
        auto load_all = [&](auto ns_tag) {
            constexpr int NS = decltype(ns_tag)::value;
#pragma unroll
            for (int e = 0; e < kFinishRegs; ++e) {
                const int f = e * 64 + lane;
                key[e] = 0ull;
                if (f < total) {
                    int sg = 0, base = 0;
#pragma unroll
                    for (int t = 0; t + 1 < NS; ++t)
                        if (t + 1 < nseg && f >= bnd[t]) { sg = t + 1; base = bnd[t]; }
                    key[e] = ckey(seg_ptr(sg)[f - base]);
                }
            }
        };
        if (nseg <= 4) load_all(std::integral_constant<int, 4>{});
        else load_all(std::integral_constant<int, 2 * kMaxSplits>{});
#pragma unroll
        for (int e = 0; e < kFinishRegs; ++e) {
            if (e * 64 + lane < total) {
                mx = key[e] > mx ? key[e] : mx;
                mn = key[e] < mn ? key[e] : mn;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a = __shfl_xor(mx, o, 64), b = __shfl_xor(mn, o, 64);
            mx = a > mx ? a : mx;
            mn = b < mn ? b : mn;
        }
        int shift = 64 - (mx == mn ? 64 : __builtin_clzll(mx ^ mn));  // bits below the shared prefix
        if (shift < 8) shift = 8;
        uint64_t prefix = mx & prefix_mask(shift);
        int kept = total;
        auto eachr = [&](auto&& fn) {
#pragma unroll
            for (int e = 0; e < kFinishRegs; ++e)
                if (e * 64 + lane < total) fn(key[e]);
        };
        if (total > kFinishCap) radix_prefix(eachr, k, kFinishCap, hist, prefix, shift, kept);
        const uint64_t pmask = prefix_mask(shift);
        int m = 0;
#pragma unroll
        for (int e = 0; e < kFinishRegs; ++e) {
            const bool take = e * 64 + lane < total && (key[e] & pmask) >= prefix;
            const uint64_t bm = __ballot(take);
            const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                    static_cast<uint32_t>(bm >> 32),
                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
            if (take && pos < kFinishCap)
                keep[pos] = Cand{v2::okey_inv(static_cast<uint32_t>(key[e] >> 32)), ~static_cast<uint32_t>(key[e])};
            m += __popcll(bm);
        }
        if (m > kFinishCap) m = kFinishCap;  // cannot happen: the prefix bounds it
        wave_lds_sync();
        finish_sort<2>(keep, m, k, os, oi, id_offset);
        return;
    }

    // streaming path: radix select on the composite key until <= kFinishCap entries remain
    uint64_t prefix = 0;
    int shift = 64, kept = total;
    if (total > kFinishCap) radix_prefix(each, k, kFinishCap, hist, prefix, shift, kept);
    // collect entries with key >= prefix (lower bits zero) into LDS, in any order
    const uint64_t pmask = prefix_mask(shift);
    int m = 0;
    for (int sg = 0; sg < nseg; ++sg) {
        const int n = __shfl(cnt, sg, 64);
        const Cand* p = seg_ptr(sg);
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            Cand c{-INFINITY, kEmptyId};
            bool take = false;
            if (i < n) {
                c = p[i];
                take = (ckey(c) & pmask) >= prefix;
            }
            const uint64_t bm = __ballot(take);
            const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                    static_cast<uint32_t>(bm >> 32),
                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
            if (take && pos < kFinishCap) keep[pos] = c;
            m += __popcll(bm);
        }
    }
    if (m > kFinishCap) m = kFinishCap;  // cannot happen: the prefix bounds it
    wave_lds_sync();
    finish_sort<2>(keep, m, k, os, oi, id_offset);
}

// per query: the rank-th largest (1-based, rank <= 32) of the union of
// n_lists (<= 64) sorted 32-entry lists (list l of query q at lists[l *
// list_stride + q * 32]) -> thr[q] (-FLT_MAX when the union has fewer finite
// entries: a running threshold), and/or the union's 32 largest, sorted, ->
// top[q * 32]. A W-lane group per query (W = 16 for <= 16 lists, else 64),
// 256 / W queries per block: the group's lists are staged in LDS, lane l
// holds the head of list l, and each round takes the group maximum (log2 W
// shuffles) and advances the winning head — rank rounds of a k-way merge
// instead of sorting all n_lists * 32 values.
template <int W>
__global__ __launch_bounds__(256) void flatip_topk_v4_threshold(const float* __restrict__ lists, int n_lists,
                                                                int64_t list_stride, int64_t nq, int rank,
                                                                float* __restrict__ thr, float* __restrict__ top) {
    constexpr int QB = 256 / W;                            // queries per block
    __shared__ float stage[QB][W][kSampleList + 1];        // [query in block][list][entry] (+1: bank spread)
    const int t = threadIdx.x, g = t / W, l = t % W;
    const int64_t q0 = static_cast<int64_t>(blockIdx.x) * QB;
    // coalesced staging: for each list, the block's QB queries x 32 entries are contiguous
    // (only the n_lists real lists; lanes past them start exhausted)
    for (int e = t; e < n_lists * QB * kSampleList; e += 256) {
        const int li = e / (QB * kSampleList), r = e - li * (QB * kSampleList), qi = r / kSampleList,
                  j = r - qi * kSampleList;
        stage[qi][li][j] =
            q0 + qi < nq ? lists[static_cast<int64_t>(li) * list_stride + (q0 + qi) * kSampleList + j] : -INFINITY;
    }
    __syncthreads();
    const int64_t q = q0 + g;
    int h = l < n_lists ? 0 : kSampleList;
    float v = l < n_lists ? stage[g][l][0] : -INFINITY;
    const int rounds = top ? kSampleList : rank;
    float kth = -INFINITY;
    const int base = (t & 63) & ~(W - 1);  // the group's first lane within the wave
    constexpr uint64_t kGroupMask = W == 64 ? ~0ull : (1ull << W) - 1;
    for (int it = 0; it < rounds; ++it) {
        float m = v;
#pragma unroll
        for (int o = W / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, W));
        const uint64_t eq = (__ballot(v == m) >> base) & kGroupMask;
        if (eq && l == __builtin_ctzll(eq)) {  // eq == 0 only for an all-NaN group: no head moves
            ++h;
            v = h < kSampleList ? stage[g][l][h] : -INFINITY;
        }
        if (it == rank - 1) kth = m;
        if (top && l == 0 && q < nq) top[q * kSampleList + it] = m;
    }
    if (thr && l == 0 && q < nq) thr[q] = kth > -FLT_MAX ? kth : -FLT_MAX;
}

inline int launch_threshold(const float* lists, int n_lists, int64_t list_stride, int64_t nq, int rank, float* thr,
                            float* top, hipStream_t st) {
    if (n_lists < 1 || n_lists > 64) return RT_ERR_UNSUPPORTED;
    if (n_lists <= 16)
        hipLaunchKernelGGL(flatip_topk_v4_threshold<16>, dim3(static_cast<unsigned>((nq + 15) / 16)), dim3(256), 0, st,
                           lists, n_lists, list_stride, nq, rank, thr, top);
    else
        hipLaunchKernelGGL(flatip_topk_v4_threshold<64>, dim3(static_cast<unsigned>((nq + 3) / 4)), dim3(256), 0, st,
                           lists, n_lists, list_stride, nq, rank, thr, top);
    return check_launch("flatip_topk_v4_threshold");
}

template <typename T, int S, int QS>
int launch_scan(const Args& a, int q_tiles, int splits, int64_t items_per_split, int stride, int rank, int* meta,
                int mode, int* fail, hipStream_t st) {
    dim3 grid(static_cast<unsigned>(q_tiles * splits));
    if (a.excl)
        hipLaunchKernelGGL((flatip_topk_v4_scan<T, S, QS, true>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split, stride, rank, meta, mode, fail);
    else
        hipLaunchKernelGGL((flatip_topk_v4_scan<T, S, QS, false>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split, stride, rank, meta, mode, fail);
    return check_launch("flatip_topk_v4_scan");
}

inline int launch_finish(const Args& a, int splits, int64_t q_pad, int mode, int* fail, hipStream_t st) {
    hipLaunchKernelGGL(flatip_topk_v4_finish<4>, dim3(static_cast<unsigned>((a.nq + 3) / 4)), dim3(256), 0, st,
                       a.cand, a.meta, splits, q_pad, a.nq, a.k, a.out_s, a.out_i, a.id_offset, mode, fail);
    return check_launch("flatip_topk_v4_finish");
}

// presampled joint threshold (several splits): a sample-only scan of every
// split (mode 3), the per-query threshold from the union of the split lists,
// the main scan against it (mode 4), the finish with the union check (mode
// 1), then the rescue pair (mode 2) — every block samples its own split only
// (the mode-1 scan has every block sample the whole corpus)
template <typename T, int S, int QS>
int launch_presampled(const Args& a, int q_tiles, int splits, int64_t items_per_split, int stride, int rank,
                      float* lists, float* thr, int* fail, hipStream_t st) {
    const int64_t q_pad = static_cast<int64_t>(q_tiles) * Geo<QS>::QT;
    Args b = a;
    b.lists_out = lists;
    int rc = launch_scan<T, S, QS>(b, q_tiles, splits, items_per_split, stride, rank, a.meta, 3, nullptr, st);
    if (rc) return rc;
    if ((rc = launch_threshold(lists, splits, q_pad * kSampleList, a.nq, rank, thr, nullptr, st))) return rc;
    b.lists_out = nullptr;
    b.thr_in = thr;
    if ((rc = launch_scan<T, S, QS>(b, q_tiles, splits, items_per_split, stride, rank, a.meta, 4, nullptr, st)))
        return rc;
    if ((rc = launch_finish(a, splits, q_pad, 1, fail, st))) return rc;
    if ((rc = launch_scan<T, S, QS>(a, q_tiles, splits, items_per_split, stride, rank, a.meta, 2, fail, st))) return rc;
    return launch_finish(a, splits, q_pad, 2, fail, st);
}

template <typename T, int S, int QS>
int launch_S(const Args& a, int q_tiles, int splits, int64_t items_per_split, int stride, int rank, int* meta,
             int* fail, hipStream_t st) {
    // joint threshold (several splits): scan + finish, then the rescue pair,
    // whose blocks exit at once unless the finish flagged one of their queries
    const int passes = fail ? 2 : 1;
    const int64_t q_pad = static_cast<int64_t>(q_tiles) * Geo<QS>::QT;
    for (int pass = 0; pass < passes; ++pass) {
        const int mode = fail ? 1 + pass : 0;
        dim3 grid(static_cast<unsigned>(q_tiles * splits));
        if (a.excl)
            hipLaunchKernelGGL((flatip_topk_v4_scan<T, S, QS, true>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                               items_per_split, stride, rank, meta, mode, fail);
        else
            hipLaunchKernelGGL((flatip_topk_v4_scan<T, S, QS, false>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                               items_per_split, stride, rank, meta, mode, fail);
        int rc = check_launch("flatip_topk_v4_scan");
        if (rc) return rc;
        hipLaunchKernelGGL(flatip_topk_v4_finish<4>, dim3(static_cast<unsigned>((a.nq + 3) / 4)), dim3(256), 0, st,
                           a.cand, meta, splits, q_pad, a.nq, a.k, a.out_s, a.out_i, a.id_offset, mode, fail);
        rc = check_launch("flatip_topk_v4_finish");
        if (rc) return rc;
    }
    return 0;
}

}  // namespace v4
}  // namespace topk
}  // namespace rt
