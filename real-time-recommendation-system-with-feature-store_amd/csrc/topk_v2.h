// Flat-IP top-K for 16-bit corpora (f16 / bf16) and k <= 128 — the C4 shape
// (65,536 queries x a 125,000-row shard, d = 128, k = 100). Included by
// topk_impl.h; same contract as flatip_topk_kernel there.
//
// * block = 8 waves (2 per SIMD, so one wave's selection overlaps the other's
//   MFMAs), 32 queries per wave held as MFMA B fragments in registers; item
//   rows stream through a double-buffered LDS tile (one barrier per 64 rows)
//   and are read as A fragments of v_mfma_f32_32x32x16_{f16,bf16}.
// * selection: per query a candidate buffer of kCap entries in global memory,
//   split in two halves owned by the two lanes that hold the query (lane and
//   lane^32 see different rows of each sub-tile), so an append is one masked
//   store at the lane's own counter — no atomics, no cross-lane slot math. Hot
//   filter per lane = max of its 16 scores against the query's threshold; a
//   sub-tile whose wave has no passing lane costs ~12 VALU.
// * item tiles arrive by LDS-DMA (global_load_lds_dwordx4, inline asm: no VGPR
//   destination) into a lane-linear image whose 16-byte chunks are XOR-swizzled
//   per row through the SOURCE address, so the A-fragment ds_read_b128 are
//   conflict-free; the next tile's DMA is issued at the top of an iteration and
//   waited for before the raw barrier at its end with a vmcnt bound derived
//   from the (wave-uniform) number of candidate stores issued after it — never
//   a blanket vmcnt(0), so appends' store acknowledgements are not waited for.
// * compaction when a buffer nears capacity: a two-pass 8-bit radix select on
//   order-preserving keys (per-wave LDS histogram) finds a 16-bit key prefix T
//   with >= k entries at or above it; entries below T can never reach the top
//   k and are dropped, and T becomes the new threshold (filter v >= thr).
//   Exact ties (more than kCap-64 entries sharing the prefix) fall back to an
//   exact register sort keeping the k best by (score desc, id asc) and a strict
//   threshold (items arrive in increasing id order, so equal later scores lose).
// * end of scan: one more compaction if needed, then a register bitonic sort
//   (128 or 512 entries) and the k best written in Faiss order.
#pragma once

namespace rt {
namespace topk {
namespace v2 {

constexpr int kWavesB = 8;            // waves per block
constexpr int kQT = 32 * kWavesB;     // queries per block
constexpr int kNT = 128;              // split granularity; items per LDS stage: Cfg2::NT
#ifndef RT_TOPK_CAP
#define RT_TOPK_CAP 512
#endif
constexpr int kCap = RT_TOPK_CAP;     // candidate entries per query
constexpr int kHalf = kCap / 2;       // per owning lane
constexpr int kE = kCap / 64;         // entries per lane in a compaction
constexpr int kMaxKv2 = 128;
#ifndef RT_TOPK_NBUF
#define RT_TOPK_NBUF 3
#endif
#ifdef RT_TOPK_PROBE_TIMING
// probe builds only: per-wave cycle attribution [total, DMA wait, barrier, appends, compaction, final]
__device__ uint64_t probe_cycles[65536 * 6];
inline void* probe_cycles_addr() {
    void* p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(probe_cycles));
    return p;
}
#define RT_PT(...) __VA_ARGS__
#else
#define RT_PT(...)
#endif
constexpr int kNBuf = RT_TOPK_NBUF;  // LDS ring depth: item tiles kNBuf-1 stages ahead (MALL latency)
static_assert(kNBuf == 2 || kNBuf == 3, "VMEM bookkeeping covers rings of 2 or 3 tiles");

// order-preserving key of a score; -0 is folded onto +0 (they compare equal)
__device__ __forceinline__ uint32_t okey(float s) {
    const float c = s + 0.0f;
    const uint32_t u = __float_as_uint(c);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float okey_inv(uint32_t k) {
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __uint_as_float(u);
}

// One 8-bit radix step over the selected keys: the bin (of (key >> shift) & 255)
// holding the kk-th largest selected key, and how many selected keys lie in
// strictly higher bins. Whole wave calls; hist = this wave's 256 LDS words.
__device__ inline void radix_bin(uint32_t* hist, const uint32_t (&key)[kE], const bool (&sel)[kE], int shift,
                                 int kk, int& bin, int& above) {
    const int lane = threadIdx.x & 63;
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < kE; ++e)
        if (sel[e]) atomicAdd(&hist[(key[e] >> shift) & 255u], 1u);
    wave_lds_sync();
    const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
    const int c4 = static_cast<int>(h.x + h.y + h.z + h.w);
    int suf = c4;  // inclusive suffix sum over lanes >= lane (bins ascend with lane)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += t;
    }
    const int ab = suf - c4;
    const int c3 = ab + static_cast<int>(h.w), c2 = c3 + static_cast<int>(h.z), c1 = c2 + static_cast<int>(h.y);
    const int c0 = c1 + static_cast<int>(h.x);
    const bool hit = ab < kk && c0 >= kk;
    const uint64_t m = __ballot(hit);
    const int src = m ? __builtin_ctzll(m) : 63;
    const int bl = c3 >= kk ? 3 : c2 >= kk ? 2 : c1 >= kk ? 1 : 0;
    const int al = c3 >= kk ? ab : c2 >= kk ? c3 : c1 >= kk ? c2 : c1;
    bin = __shfl(4 * lane + bl, src, 64);
    above = __shfl(al, src, 64);
    wave_lds_sync();
}

// entry idx of a query buffer holding n0 entries in its first half and the
// rest in its second
__device__ __forceinline__ const Cand& entry(const Cand* buf, int n0, int idx) {
    return idx < n0 ? buf[idx] : buf[kHalf + (idx - n0)];
}

// Shrink one query's buffer (halves of n0 and n1 entries, k <= n0+n1) to a
// superset of its top k, re-dealt over the halves (entry j → half j&1, slot
// j>>1). Returns the new total; thr = the new filter threshold (v >= thr).
__device__ __noinline__ int compact_query(Cand* __restrict__ buf, int n0, int n1, int k, uint32_t* hist,
                                          float& thr) {
    const int lane = threadIdx.x & 63;
    const int n = n0 + n1;
    float s[kE];
    uint32_t id[kE], key[kE];
    bool sel[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const int idx = e * 64 + lane;
        sel[e] = idx < n;
        const Cand c = sel[e] ? entry(buf, n0, idx) : Cand{-INFINITY, kEmptyId};
        s[e] = c.s;
        id[e] = c.i;
        key[e] = okey(c.s);
    }
    int b1, a1, b2, a2;
    radix_bin(hist, key, sel, 24, k, b1, a1);
    bool sel2[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) sel2[e] = sel[e] && (key[e] >> 24) == static_cast<uint32_t>(b1);
    radix_bin(hist, key, sel2, 16, k - a1, b2, a2);
    const uint32_t T = (static_cast<uint32_t>(b1) << 24) | (static_cast<uint32_t>(b2) << 16);
    bool keep[kE];
    int total = 0;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        keep[e] = sel[e] && key[e] >= T;
        total += __popcll(__ballot(keep[e]));
    }
    if (total <= kCap - 64) {
        int base = 0;
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            const uint64_t m = __ballot(keep[e]);
            const int pos = base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
            if (keep[e]) buf[(pos & 1) * kHalf + (pos >> 1)] = Cand{s[e], id[e]};
            base += __popcll(m);
        }
        thr = T <= 0x007FFFFFu ? -INFINITY : okey_inv(T);  // bin of -inf / NaN keys: admit all
        __threadfence_block();
        return total;
    }
    // massive exact ties: exact sort, keep the k best, strict threshold
#pragma unroll
    for (int e = 0; e < kE; ++e)
        if (!sel[e]) { s[e] = -INFINITY; id[e] = kEmptyId; }
    wave_sort_regs<kE>(s, id);
    float kth = -INFINITY;
#pragma unroll
    for (int j = 0; j < kE; ++j) {
        const int r = lane * kE + j;
        if (r < k) buf[(r & 1) * kHalf + (r >> 1)] = Cand{s[j], id[j]};
        if (r == k - 1) kth = s[j];
    }
    kth = __shfl(kth, (k - 1) / kE, 64);
    thr = nextafterf(kth, INFINITY);
    __threadfence_block();
    return k;
}

// Sort one query's buffer (halves of n0 / n1 entries, n0+n1 <= 64*E) and
// write its k best.
template <int E>
__device__ __noinline__ void emit_sorted(const Cand* __restrict__ buf, int n0, int n1, int k,
                                         float* __restrict__ os, int64_t* __restrict__ oi, int64_t id_offset) {
    const int lane = threadIdx.x & 63;
    const int n = n0 + n1;
    float s[E];
    uint32_t id[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int r = lane * E + j;
        const Cand c = r < n ? entry(buf, n0, r) : Cand{-INFINITY, kEmptyId};
        s[j] = c.s;
        id[j] = c.i;
    }
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// wait until at most n (wave-uniform, >= 0) vector-memory operations are in
// flight — exactly n (capped at the counter's 63): a bound rounded down would
// also wait for the youngest candidate stores' acknowledgements
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
__device__ __forceinline__ void wait_vm_le(int n) { wait_vm_range<0, 63>(n > 63 ? 63 : n); }

template <typename T, int S>
struct Cfg2 {
    static constexpr int KK = Mfma<T>::kK;                      // k per MFMA: 16 (f16/bf16), 2 (f32)
    static constexpr int DP = S * KK;                            // padded d
    static constexpr int VEC = 16 / static_cast<int>(sizeof(T));  // 8 elements per 16 B
    static constexpr int ROWB = DP * static_cast<int>(sizeof(T));   // bytes per LDS row (unpadded)
    static constexpr int P = ROWB / 16;                              // 16-byte chunks per row
    static constexpr int NT = ROWB <= 256 ? 128 : 64;               // items per LDS stage
    static constexpr int TILE_BYTES = NT * ROWB;
    static constexpr int DMA_PER_WAVE = TILE_BYTES / 1024 / kWavesB;  // 1 KiB per wave-instruction
    static_assert(DMA_PER_WAVE * 1024 * kWavesB == TILE_BYTES, "tile must split into whole DMA pieces");
    // chunk swizzle of row r: distinct bank groups for the 16 rows a ds_read_b128 lane group touches
    __device__ static int swz(int r) { return P >= 16 ? (r & 15) : ((r / (16 / P)) & (P - 1)); }
};

static __device__ const uint4 kZero16 = {0u, 0u, 0u, 0u};

template <typename P>
__device__ __forceinline__ uint32_t lds_addr(P* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)(p)));
}
// one LDS-DMA piece: each lane's 16 bytes from gsrc land at lds_dst + 16 * lane
// (M0 carries the wave-uniform destination; saved and restored in the statement)
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// grid: 1-D, block b → (query tile b / splits, item split b % splits); with
// splits | 8 every XCD (b mod 8) streams one split of the corpus.
template <typename T, int S, bool EXCL>
__global__ __launch_bounds__(512) void flatip_topk_v2_kernel(Args a, int splits, int64_t items_per_split) {
    using M = Mfma<T>;
    using C = Cfg2<T, S>;
    constexpr int DP = C::DP, VEC = C::VEC, ROWB = C::ROWB;
    __shared__ __attribute__((aligned(1024))) T tile[kNBuf][C::TILE_BYTES / sizeof(T)];
    __shared__ __attribute__((aligned(16))) uint32_t hist[kWavesB][256];

    const T* __restrict__ Q = reinterpret_cast<const T*>(a.Q);
    const T* __restrict__ X = reinterpret_cast<const T*>(a.X);
    const int d = a.d, k = a.k;
    const int64_t nq = a.nq;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 31, half = lane >> 5;
    const int split = static_cast<int>(blockIdx.x % static_cast<unsigned>(splits));
    const int64_t qtile = blockIdx.x / static_cast<unsigned>(splits);
    const int64_t qw = qtile * kQT + wave * 32;  // wave's first query
    const int64_t q = qw + col;
    const bool qok = q < nq;
    const int64_t i_begin = static_cast<int64_t>(split) * items_per_split;
    const int64_t i_end = (i_begin + items_per_split) < a.nx ? (i_begin + items_per_split) : a.nx;
    const int row_vecs = d / VEC;
    const int64_t q_pad = static_cast<int64_t>(gridDim.x / splits) * kQT;  // buffers per split
    Cand* const cbase = a.cand + (static_cast<int64_t>(split) * q_pad + qw) * kCap;  // wave's 32 buffers
    uint32_t* const whist = hist[wave];

    typename M::frag qf[S];
    {
        const T* qrow = Q + (qok ? q : 0) * d;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k0 = (C::KK == 2) ? 2 * s + half : 16 * s + 8 * half;
            if (qok && k0 < d) qf[s] = frag_from<T>(qrow + k0);
            else qf[s] = typename M::frag{};
        }
    }
    // drain the fragment loads here: left in flight, the loop header's merged
    // wait state would force a vmcnt(0) (and so the tile prefetch) every tile
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if constexpr (C::KK == 2) {
            asm volatile("" ::"v"(qf[s]));
        } else {
            const uint4 t = __builtin_bit_cast(uint4, qf[s]);
            asm volatile("" ::"v"(t.x), "v"(t.y), "v"(t.z), "v"(t.w));
        }
    }
    const uint32_t* excl = (EXCL && qok) ? a.excl + q * a.excl_words : nullptr;
    float thr = qok ? -FLT_MAX : INFINITY;
#ifdef RT_TOPK_PROBE_NOSEL
    thr = INFINITY;  // probe builds only (tools/hip_probe/topk_probe.hip): the scan without selection
#endif
    // append cursor: byte offset of the lane's next entry from the wave's
    // (uniform) buffer base, so a store is SADDR + one 32-bit VGPR
    // (readfirstlane returns int: take each half as uint32_t before widening, or a
    // low word with bit 31 set sign-extends over the high word)
    const uint32_t wb_lo = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase))));
    const uint32_t wb_hi = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase) >> 32)));
    const uint64_t wbase = (static_cast<uint64_t>(wb_hi) << 32) | wb_lo;
    const uint32_t woff0 = static_cast<uint32_t>((col * kCap + half * kHalf) * sizeof(Cand));
    uint32_t woff = woff0;
    // compaction trigger per lane: a full half, or (small k) once enough entries
    // arrived to refresh a stale threshold
#ifndef RT_TOPK_LIM_MUL
#define RT_TOPK_LIM_MUL 0
#endif
#ifndef RT_TOPK_LIM_ADD
#define RT_TOPK_LIM_ADD 32
#endif
    const int lim_n = RT_TOPK_LIM_MUL > 0 ? min(kHalf - 16, RT_TOPK_LIM_MUL * k + RT_TOPK_LIM_ADD) : kHalf - 16;
    const uint32_t woff_lim = woff0 + static_cast<uint32_t>(lim_n * sizeof(Cand));

    // LDS-DMA of one tile (rows t0 .., zero chunks past d; rows past the split
    // end read a clamped valid row — their scores are masked to -inf)
    // VMEM instructions issued after the DMA the end of this stage waits for
    // (vm_old: the next stage's) and after the youngest DMA (vm_new); wave-uniform.
    // A drain (compaction) zeroes both: then the waits are no-ops.
    int vm_old = 0, vm_new = 0;
    const uint32_t wave_u = __builtin_amdgcn_readfirstlane(wave);
    auto fetch = [&](int64_t t0, int buf) {
        const uint32_t base = lds_addr(&tile[buf][0]) + wave_u * (C::DMA_PER_WAVE * 1024);
#pragma unroll
        for (int j = 0; j < C::DMA_PER_WAVE; ++j) {
            const int o = (wave * C::DMA_PER_WAVE + j) * 1024 + lane * 16;
            const int r = o / ROWB;
            const int c = ((o % ROWB) >> 4) ^ C::swz(r);
            int64_t item = t0 + r;
            item = item < i_end ? item : i_end - 1;
            const void* src = c < row_vecs ? static_cast<const void*>(X + item * d + c * VEC)
                                           : static_cast<const void*>(&kZero16);
            glds16(src, base + j * 1024);
        }
        if constexpr (kNBuf == 3) vm_old += C::DMA_PER_WAVE;  // younger than the awaited DMA
        vm_new = 0;
    };
    // the next stage's DMA has landed (every VMEM operation younger than it counted)
    auto fetch_wait = [&]() { wait_vm_le(vm_old); };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // Selection from one 32-item sub-tile's scores (acc[r] = item sub0 + tile_row(r, half),
    // query col), in two parts. masks(): per score one compare into an SGPR wave
    // mask (v_cmp → s[..], no per-lane mask building) — straight-line, so the
    // 16-bit loop below runs it in the MFMA gaps of the next sub-tile. appends():
    // the wave visits only the rows r some lane passes and stores those lanes'
    // entries with two masked dword stores per row.
    auto masks = [&](const f32x16& acc, uint64_t (&pm)[16], uint64_t& any) {
        any = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            pm[r] = __ballot(acc[r] >= thr);
            any |= pm[r];
        }
    };
    auto appends = [&](const f32x16& acc, int64_t sub0, const uint64_t (&pm)[16], uint64_t any) {
        if (!any) return;
        uint32_t xw = 0u;
        if constexpr (EXCL) {
            if (excl) xw = excl[sub0 >> 5];  // sub0 is 32-aligned: one bitmap word per sub-tile
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (pm[r]) {  // wave-uniform
                bool p;
                if constexpr (EXCL) {
                    p = acc[r] >= thr && !((xw >> tile_row(r, half)) & 1u);
                    if (!__ballot(p)) continue;
                } else {
                    p = __builtin_amdgcn_inverse_ballot_w64(pm[r]);  // exec = pm[r], no compare
                }
                vm_old += 2;  // exactly two store instructions for the wave
                vm_new += 2;
                if (p) {
                    // score and id as two dword stores of one entry (SADDR form: uniform base +
                    // 32-bit lane offset), no register moves to pair them up; the cursor
                    // advances inside the statement (under this exec mask, in place)
                    const uint32_t id = static_cast<uint32_t>(sub0 + tile_row(r, half));
                    asm volatile(
                        "global_store_dword %0, %1, %2\n\tglobal_store_dword %0, %3, %2 offset:4\n\t"
                        "v_add_u32 %0, 8, %0"
                        : "+v"(woff)
                        : "v"(acc[r]), "s"(wbase), "v"(id)
                        : "memory");
                }
            }
        }
    };
    auto select = [&](const f32x16& acc, int64_t sub0) {
        uint64_t pm[16], any;
        masks(acc, pm, any);
        appends(acc, sub0, pm, any);
    };
    // compact every buffer of this wave that may overflow on the next sub-tile
    auto maybe_compact = [&]() {
        const uint64_t m = __ballot(woff > woff_lim);
        uint32_t need = static_cast<uint32_t>(m) | static_cast<uint32_t>(m >> 32);
        if (!need) return;
        __threadfence_block();
        while (need) {
            const int c = __builtin_ctz(need);
            need &= need - 1;
            const int cnt = static_cast<int>((woff - woff0) / sizeof(Cand));
            const int n0 = __shfl(cnt, c, 64), n1 = __shfl(cnt, c + 32, 64);
            float nt;
            const int nn = compact_query(cbase + static_cast<int64_t>(c) * kCap, n0, n1, k, whist, nt);
            if (col == c) {
                woff = woff0 + static_cast<uint32_t>((half ? nn >> 1 : (nn + 1) >> 1) * sizeof(Cand));
                thr = nt;
            }
        }
        vm_old = vm_new = 0;  // the compaction drained every outstanding VMEM operation
    };

    constexpr int NT = C::NT;
    // prologue: stages 0 .. kNBuf-2 in flight, stage 0 landed
#pragma unroll
    for (int b = 0; b < kNBuf - 1; ++b)
        if (i_begin + b * NT < i_end) fetch(i_begin + b * NT, b);
    wait_vm_le(0);
    vm_old = vm_new = 0;
    raw_barrier();
    RT_PT(uint64_t pc_wait = 0, pc_bar = 0, pc_app = 0, pc_cmp = 0; const uint64_t pc_start = clock64();)
    int cur = 0;
    auto next_stage = [&]() {
        // next stage: the DMA its end waits for is the youngest one now (kNBuf = 3);
        // for kNBuf = 2 that DMA is issued at its top (fetch adds its count)
        vm_old = kNBuf == 2 ? 0 : vm_new;
        cur = cur == kNBuf - 1 ? 0 : cur + 1;
    };
    auto mask_tail = [&](f32x16& acc, int64_t sub0) {
        if (sub0 + 32 > i_end) {  // rows past the end never qualify
            const int left = static_cast<int>(i_end - sub0);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (tile_row(r, half) >= left) acc[r] = -INFINITY;
        }
    };
    // fp32, and 16-bit d > 128 (16-bit d <= 128 runs topk_v3.h)
    for (int64_t t0 = i_begin; t0 < i_end; t0 += NT) {
        const T* tl = tile[cur];
        const bool more = t0 + NT < i_end;
        // stage + kNBuf-1 into the buffer read in the previous stage (all waves are past its barrier)
        if (t0 + (kNBuf - 1) * NT < i_end) fetch(t0 + (kNBuf - 1) * NT, cur == 0 ? kNBuf - 1 : cur - 1);
#pragma unroll
        for (int rt = 0; rt < NT / 32; ++rt) {
            const int64_t sub0 = t0 + rt * 32;
            if (sub0 >= i_end) break;  // block-uniform
            f32x16 acc = {};
            const int row = rt * 32 + col;
            const T* arow = tl + row * DP;
            if constexpr (C::KK == 2) {
                // f32: k-step s takes element 2s + half (natural k order: the MFMA chain
                // is the oracle's sequential fmaf order); one b128 read serves 2 steps
#pragma unroll
                for (int j = 0; j < S / 2; ++j) {
                    const float4 v = *reinterpret_cast<const float4*>(arow + (j ^ C::swz(row)) * VEC);
                    acc = M::run(half ? v.y : v.x, qf[2 * j], acc);
                    acc = M::run(half ? v.w : v.z, qf[2 * j + 1], acc);
                }
            } else {
                typename M::frag af[S];
#pragma unroll
                for (int s = 0; s < S; ++s)
                    af[s] = frag_from<T>(arow + ((2 * s + half) ^ C::swz(row)) * VEC);
                __builtin_amdgcn_sched_barrier(0);  // every read in flight before the first MFMA waits
#pragma unroll
                for (int s = 0; s < S; ++s) acc = M::run(af[s], qf[s], acc);
            }
            mask_tail(acc, sub0);
            select(acc, sub0);
            maybe_compact();
        }
        RT_PT(uint64_t c0 = clock64();)
        if (more) fetch_wait();
        RT_PT(uint64_t c1 = clock64(); pc_wait += c1 - c0;)
        raw_barrier();
        RT_PT(pc_bar += clock64() - c1;)
        next_stage();
    }

    RT_PT(uint64_t c4 = clock64();)
    // ---- final selection, one query of the wave at a time ----
    __threadfence_block();
    float* os = a.out_s + static_cast<int64_t>(split) * nq * k;
    int64_t* oi = a.out_i + static_cast<int64_t>(split) * nq * k;
    for (int c = 0; c < 32; ++c) {
        const int64_t gq = qw + c;
        if (gq >= nq) break;
        Cand* b = cbase + static_cast<int64_t>(c) * kCap;
        const int cnt = static_cast<int>((woff - woff0) / sizeof(Cand));
        int n0 = __shfl(cnt, c, 64), n1 = __shfl(cnt, c + 32, 64);
        if (n0 + n1 > 128) {
            float nt;
            const int nn = compact_query(b, n0, n1, k, whist, nt);
            n0 = (nn + 1) >> 1;
            n1 = nn >> 1;
        }
        if (n0 + n1 <= 128) emit_sorted<2>(b, n0, n1, k, os + gq * k, oi + gq * k, a.id_offset);
        else emit_sorted<kE>(b, n0, n1, k, os + gq * k, oi + gq * k, a.id_offset);
    }
#ifdef RT_TOPK_PROBE_TIMING
    const uint64_t c5 = clock64();
    const int64_t gw = static_cast<int64_t>(blockIdx.x) * kWavesB + wave;
    if (lane == 0 && gw < 65536) {
        uint64_t* o = probe_cycles + gw * 6;
        o[0] = c5 - pc_start; o[1] = pc_wait; o[2] = pc_bar; o[3] = pc_app; o[4] = pc_cmp; o[5] = c5 - c4;
    }
#endif
}

inline int planned_splits(int64_t q_tiles, int64_t nx) {
    // ~1 block (8 waves) per CU (fewer splits = fewer early-phase appends);
    // every split >= 2 LDS stages, so small corpora still fill the chip
    int64_t splits = (256 + q_tiles - 1) / q_tiles;
    int64_t max_splits = (nx + 2 * kNT - 1) / (2 * kNT);
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    // powers of two up to 8 keep one split per XCD
    int64_t p = 1;
    while (p * 2 <= splits && p < 8) p *= 2;
    if (splits > 8) p = splits;
    return static_cast<int>(p > 64 ? 64 : p);
}

template <typename T, int S>
int launch_S(const Args& a, int splits, int64_t items_per_split, hipStream_t st) {
    const int64_t q_tiles = (a.nq + kQT - 1) / kQT;
    dim3 grid(static_cast<unsigned>(q_tiles * splits));
    if (a.excl)
        hipLaunchKernelGGL((flatip_topk_v2_kernel<T, S, true>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split);
    else
        hipLaunchKernelGGL((flatip_topk_v2_kernel<T, S, false>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split);
    return check_launch("flatip_topk_v2_kernel");
}

}  // namespace v2
}  // namespace topk
}  // namespace rt
