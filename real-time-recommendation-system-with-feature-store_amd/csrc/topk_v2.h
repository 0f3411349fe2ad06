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
constexpr int kCap = 512;             // candidate entries per query
constexpr int kHalf = kCap / 2;       // per owning lane
constexpr int kE = kCap / 64;         // entries per lane in a compaction
constexpr int kMaxKv2 = 128;

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
template <int E = kE>
__device__ inline void radix_bin(uint32_t* hist, const uint32_t (&key)[E], const bool (&sel)[E], int shift,
                                 int kk, int& bin, int& above) {
    const int lane = threadIdx.x & 63;
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < E; ++e)
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
template <int HALF = kHalf>
__device__ __forceinline__ const Cand& entry(const Cand* buf, int n0, int idx) {
    return idx < n0 ? buf[idx] : buf[HALF + (idx - n0)];
}

// Shrink one query's buffer (halves of n0 and n1 entries, k <= n0+n1) to a
// superset of its top k, re-dealt over the halves (entry j → half j&1, slot
// j>>1). Returns the new total; thr = the new filter threshold (v >= thr).
// CAP = the buffer's entry capacity (v2/v3: kCap; v4: its own).
template <int CAP = kCap>
__device__ __forceinline__ int compact_query_body(Cand* __restrict__ buf, int n0, int n1, int k, uint32_t* hist,
                                                  float& thr) {
    constexpr int kE = CAP / 64, kHalf = CAP / 2, kCap = CAP;
    const int lane = threadIdx.x & 63;
    const int n = n0 + n1;
    float s[kE];
    uint32_t id[kE], key[kE];
    bool sel[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const int idx = e * 64 + lane;
        sel[e] = idx < n;
        const Cand c = sel[e] ? entry<kHalf>(buf, n0, idx) : Cand{-INFINITY, kEmptyId};
        s[e] = c.s;
        id[e] = c.i;
        key[e] = okey(c.s);
    }
    int b1, a1, b2, a2;
    radix_bin<kE>(hist, key, sel, 24, k, b1, a1);
    bool sel2[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) sel2[e] = sel[e] && (key[e] >> 24) == static_cast<uint32_t>(b1);
    radix_bin<kE>(hist, key, sel2, 16, k - a1, b2, a2);
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
// out of line (v2/v3 scans: keeps the compaction's registers out of the loop)
template <int CAP = kCap>
__device__ __noinline__ int compact_query(Cand* __restrict__ buf, int n0, int n1, int k, uint32_t* hist,
                                          float& thr) {
    return compact_query_body<CAP>(buf, n0, n1, k, hist, thr);
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
// flight, rounded down to a power of two
__device__ __forceinline__ void wait_vm_le(int n) {
    if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

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
    __shared__ __attribute__((aligned(1024))) T tile[2][C::TILE_BYTES / sizeof(T)];
    __shared__ __attribute__((aligned(16))) uint32_t hist[kWavesB][256];
    __shared__ __attribute__((aligned(16))) float scr[kWavesB * 64 * 20];  // per-lane score rows (80 B: conflict-free b128)

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
    Cand* const mybuf = cbase + static_cast<int64_t>(col) * kCap + half * kHalf;  // this lane's half
    uint32_t* const whist = hist[wave];
    float* const wscr = scr + (wave * 64 + lane) * 20;

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
    int cnt = 0;

    // LDS-DMA of one tile (rows t0 .., zero chunks past d; rows past the split
    // end read a clamped valid row — their scores are masked to -inf)
    int vm_after = 0;  // VMEM instructions issued since the last DMA (wave-uniform); >= 1<<20: drained
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
        vm_after = 0;
    };
    // the DMA into the other buffer has landed (its count bound is exact or drained)
    auto fetch_wait = [&]() {
        if (vm_after < (1 << 20)) wait_vm_le(vm_after);
    };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // select from one 32-item sub-tile's scores (acc[r] = item sub0 + tile_row(r, half), query col)
    auto select = [&](const f32x16& acc, int64_t sub0) {
        float m = acc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, acc[r]);
        if (__ballot(m >= thr) == 0) return;
        // per-lane pass mask, 2 VALU per score: bit 15-r <=> acc[r] passes
        uint32_t bits = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            asm("v_cmp_ge_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
                : "+v"(bits)
                : "v"(acc[r]), "v"(thr)
                : "vcc");
        if constexpr (EXCL) {
            if (excl) {
                const uint32_t xw = excl[sub0 >> 5];  // sub0 is 32-aligned: one bitmap word per sub-tile
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if ((xw >> tile_row(r, half)) & 1u) bits &= ~(1u << (15 - r));
            }
        }
        // the lane's scores go through its LDS scratch row so the append loop
        // can index them; the wave loops max-popcount times (1-2 late in a scan)
        if (bits) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<float4*>(wscr + 4 * i) =
                    make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]);
        }
        wave_lds_sync();
        while (__ballot(bits != 0u)) {
            ++vm_after;  // one store instruction for the wave
            if (bits) {
                const int b = 31 - __builtin_clz(bits);  // highest set bit = lowest r
                bits &= ~(1u << b);
                const int r = 15 - b;
                const float v = wscr[r];
                mybuf[cnt] = Cand{v, static_cast<uint32_t>(sub0 + tile_row(r, half))};
                ++cnt;
            }
        }
    };
    // compact every buffer of this wave that may overflow on the next sub-tile
    auto maybe_compact = [&]() {
        const uint64_t m = __ballot(cnt > kHalf - 16);
        uint32_t need = static_cast<uint32_t>(m) | static_cast<uint32_t>(m >> 32);
        if (!need) return;
        __threadfence_block();
        while (need) {
            const int c = __builtin_ctz(need);
            need &= need - 1;
            const int n0 = __shfl(cnt, c, 64), n1 = __shfl(cnt, c + 32, 64);
            float nt;
            const int nn = compact_query(cbase + static_cast<int64_t>(c) * kCap, n0, n1, k, whist, nt);
            if (col == c) {
                cnt = half ? nn >> 1 : (nn + 1) >> 1;
                thr = nt;
            }
        }
        vm_after = 1 << 20;  // the compaction drained every outstanding VMEM operation
    };

    if (i_begin < i_end) {
        fetch(i_begin, 0);
        wait_vm_le(0);
    }
    raw_barrier();
    int cur = 0;
    constexpr int NT = C::NT;
    for (int64_t t0 = i_begin; t0 < i_end; t0 += NT) {
        const T* tl = tile[cur];
        const bool more = t0 + NT < i_end;
        // the next tile's DMA: buffer cur^1 was last read before the previous barrier
        if (more) fetch(t0 + NT, cur ^ 1);
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
                for (int s = 0; s < S; ++s) af[s] = frag_from<T>(arow + ((2 * s + half) ^ C::swz(row)) * VEC);
                __builtin_amdgcn_sched_barrier(0);  // every read in flight before the first MFMA waits
#pragma unroll
                for (int s = 0; s < S; ++s) acc = M::run(af[s], qf[s], acc);
            }
            if (sub0 + 32 > i_end) {  // rows past the end never qualify
                const int left = static_cast<int>(i_end - sub0);
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (tile_row(r, half) >= left) acc[r] = -INFINITY;
            }
            select(acc, sub0);
            maybe_compact();
        }
        if (more) fetch_wait();
        raw_barrier();
        cur ^= 1;
    }

    // ---- final selection, one query of the wave at a time ----
    __threadfence_block();
    float* os = a.out_s + static_cast<int64_t>(split) * nq * k;
    int64_t* oi = a.out_i + static_cast<int64_t>(split) * nq * k;
    for (int c = 0; c < 32; ++c) {
        const int64_t gq = qw + c;
        if (gq >= nq) break;
        Cand* b = cbase + static_cast<int64_t>(c) * kCap;
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
