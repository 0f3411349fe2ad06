// Flat-IP top-K for 16-bit corpora with d <= 128 and k <= RT_TOPK3_MAXK (32):
// the small-k C4 shapes (65,536 queries x a 125,000-row f16 shard, d = 128,
// k = 1 / 10); larger k goes to topk_v4.h (large corpora) or topk_v2.h (the
// dispatch in topk_impl.h). Included by topk_impl.h; same contract, grid, plan
// and workspace as the v2 kernel
// (topk_v2.h), whose candidate buffers, radix compaction and final sort it
// reuses. What differs is the scan, built for a low instruction count per
// 32 x 32 score sub-tile (8 MFMAs at d = 128):
//
// * LDS image: item rows at a stride of one 16-byte pad chunk past the row
//   (rows 16 B apart in banks), so the A-fragment ds_read_b128 are
//   conflict-free with NO address swizzle: a lane's fragment address is one
//   VGPR per stage plus an immediate offset (row block, k step).
// * DMA sources: SADDR form — the stage's first row in SGPRs plus a per-lane
//   32-bit offset of each 16-byte slot fixed for the scan (no address VALU);
//   only the last, partial stage clamps rows.
// * sub-tile t's MFMA chain runs with sub-tile t-1's 16 threshold compares
//   (v_cmp into SGPR wave masks) in its gaps, t+1's A fragments read into the
//   other fragment set behind it, then t-1's appends (two masked dword stores
//   per row some lane passes) and the compaction check. Scores alternate
//   between two accumulators, so nothing is copied.
// * three-stage LDS ring: tiles are DMA'd two stages ahead.
#pragma once


namespace rt {
namespace topk {
namespace v3 {

using v2::compact_query;
using v2::emit_sorted;
using v2::kCap;
using v2::kE;
using v2::kHalf;
using v2::kNT;
using v2::kQT;
using v2::kWavesB;
using v2::lds_addr;

// wait until at most n (wave-uniform, >= 0) vector-memory operations are in
// flight — exactly n (capped at the counter's 63), so no candidate store's
// acknowledgement is waited for
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

#ifdef RT_TOPK_PROBE_TIMING
// probe builds only (tools/hip_probe/topk_probe.hip): per-wave cycle attribution
// [total, DMA wait, barrier, sub-tile steps, compaction, final]
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

#ifndef RT_TOPK3_NT
#define RT_TOPK3_NT 128
#endif
#ifndef RT_TOPK3_RING
#define RT_TOPK3_RING 3
#endif
template <typename T, int S>
struct Cfg3 {
    static_assert(sizeof(T) == 2 && S <= 8, "v3: 16-bit, d <= 128");
    static constexpr int DP = S * 16;                 // padded d (elements)
    static constexpr int P = DP * 2 / 16;             // 16-byte data chunks per row
    static constexpr int RS = (P + 1) * 16;           // LDS row stride (bytes): one pad chunk
    static constexpr int NT = RT_TOPK3_NT;            // rows per stage (a multiple of 64)
    static constexpr int NSUB = NT / 32;
    static constexpr int SLOTS = NT * (P + 1);        // 16-byte slots per stage
    static constexpr int PIECES = SLOTS / 64;         // 64-slot DMA pieces (1 KiB) per stage
    static constexpr int MAXP = (PIECES + kWavesB - 1) / kWavesB;  // pieces per wave, at most
    static constexpr int TILE_BYTES = SLOTS * 16;
    static_assert(PIECES * 64 == SLOTS, "whole DMA pieces");
};
#ifndef RT_TOPK3_PAIRCMP
#define RT_TOPK3_PAIRCMP 0
#endif
#ifndef RT_TOPK3_LIMK
#define RT_TOPK3_LIMK 2
#endif
constexpr int kRefreshMul = RT_TOPK3_LIMK;
#ifndef RT_TOPK3_MAXK
#define RT_TOPK3_MAXK 32
#endif
constexpr int kMaxKv3 = RT_TOPK3_MAXK;  // larger k runs v2 (see topk_impl.h)
constexpr int kRing = RT_TOPK3_RING;  // LDS ring depth: 2 (DMA one stage ahead) or 3 (two)
static_assert(kRing >= 2 && kRing <= 4, "ring of 2..4 stages");

template <typename T, int S, bool EXCL>
__global__ __launch_bounds__(512) void flatip_topk_v3_kernel(Args a, int splits, int64_t items_per_split) {
    using M = Mfma<T>;
    using C = Cfg3<T, S>;
    typedef typename M::frag frag;
    __shared__ __attribute__((aligned(1024))) char tile[kRing][C::TILE_BYTES];
    __shared__ __attribute__((aligned(16))) uint32_t hist[kWavesB][256];
    __shared__ __attribute__((aligned(16))) float scr[kWavesB * 64 * 20];  // per-lane score rows (80 B: conflict-free b128)

    const T* __restrict__ Q = reinterpret_cast<const T*>(a.Q);
    const char* __restrict__ Xb = reinterpret_cast<const char*>(a.X);
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
    const int64_t row_bytes = static_cast<int64_t>(d) * 2;
    const int64_t q_pad = static_cast<int64_t>(gridDim.x / splits) * kQT;  // buffers per split
    Cand* const cbase = a.cand + (static_cast<int64_t>(split) * q_pad + qw) * kCap;  // wave's 32 buffers
    uint32_t* const whist = hist[wave];
    float* const wscr = scr + (wave * 64 + lane) * 20;

    frag qf[S];
    {
        const T* qrow = Q + (qok ? q : 0) * d;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k0 = 16 * s + 8 * half;
            if (qok && k0 < d) qf[s] = frag_from<T>(qrow + k0);
            else qf[s] = frag{};
        }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {  // drained here, not at the loop header's merged wait
        const uint4 t = __builtin_bit_cast(uint4, qf[s]);
        asm volatile("" ::"v"(t.x), "v"(t.y), "v"(t.z), "v"(t.w));
    }
    const uint32_t* excl = (EXCL && qok) ? a.excl + q * a.excl_words : nullptr;
    float thr = qok ? -FLT_MAX : INFINITY;
#ifdef RT_TOPK_PROBE_NOSEL
    thr = INFINITY;  // probe builds only: the scan without selection
#endif

    // append cursor (see v2): byte offset of the lane's next entry from the
    // wave's uniform buffer base; compaction once a half nears full
    const uint32_t wb_lo = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase))));
    const uint32_t wb_hi = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uint64_t>(cbase) >> 32)));
    const uint64_t wbase = (static_cast<uint64_t>(wb_hi) << 32) | wb_lo;
    const uint32_t woff0 = static_cast<uint32_t>((col * kCap + half * kHalf) * sizeof(Cand));
    uint32_t woff = woff0;
    // checked once per stage (or per pair of sub-tiles): room for the appends until the next check;
    // small k compacts early too — a half holding ~2k entries refreshes a stale threshold
    constexpr int kHead = RT_TOPK3_PAIRCMP ? 2 * 16 : C::NSUB * 16;  // appends between checks, at most
    const int lim_n = kRefreshMul > 0 ? min(kHalf - kHead, kRefreshMul * k + 32) : kHalf - kHead;
    const uint32_t woff_lim = woff0 + static_cast<uint32_t>(lim_n * sizeof(Cand));

    // ---- DMA plan: this wave's pieces w, w+8, ... of a stage ----
    // SADDR form: source = the stage's first row (uniform, SGPRs) + a 32-bit
    // per-lane offset fixed for the whole scan. Pad slots (and, for d < 16 S,
    // chunks past d) read chunk 0 of the same row: finite data that only ever
    // meets zero query fragments / is never read as a fragment.
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int npieces = (C::PIECES - wave_u + kWavesB - 1) / kWavesB;  // wave-uniform
    const int row_vecs = d / 8;
    uint32_t soff[C::MAXP];  // byte offset of this lane's slot source from the stage's first row
#pragma unroll
    for (int i = 0; i < C::MAXP; ++i) {
        const int o = (wave_u + kWavesB * i) * 64 + lane;
        const int r = o / (C::P + 1), c = o % (C::P + 1);
        soff[i] = static_cast<uint32_t>(r * static_cast<int>(row_bytes) + (c < row_vecs ? c * 16 : 0));
    }
    const uint32_t tile0 = lds_addr(&tile[0][0]);
    // VMEM bookkeeping (wave-uniform): `issued` counts this wave's vector-memory
    // operations; mk[j] = the count right after the DMA of stage s+1+j was
    // issued (mk[0]: the one the current stage's end waits for). Waiting for
    // vmcnt <= issued - mk[0] waits for that DMA and nothing younger — never for
    // candidate stores' acknowledgements. A drain sets every mark to `issued`.
    int issued = 0;
    int mk[kRing - 1];
#pragma unroll
    for (int j = 0; j < kRing - 1; ++j) mk[j] = 0;
    auto fetch = [&](int64_t t0, int buf) {
        const uint32_t base = tile0 + buf * C::TILE_BYTES + wave_u * 1024;
        const char* sb = Xb + t0 * row_bytes;
        const uint64_t sbu = reinterpret_cast<uint64_t>(sb);
        const int rem = static_cast<int>(i_end - t0 < C::NT ? i_end - t0 : C::NT);
#pragma unroll
        for (int i = 0; i < C::MAXP; ++i) {
            if (i < npieces) {
                uint32_t off = soff[i];
                if (rem < C::NT) {  // rows past the split end read its last row (masked)
                    const int r = ((wave_u + kWavesB * i) * 64 + lane) / (C::P + 1);
                    if (r >= rem) off -= static_cast<uint32_t>((r - (rem - 1)) * row_bytes);
                }
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
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

    // ---- selection ----
    // Per lane (= per query, per half of the sub-tile's rows): a max-of-16
    // filter against the query's threshold (most sub-tiles stop at the wave
    // ballot); otherwise a 16-bit pass mask (2 VALU per score), the lane's scores
    // staged in its LDS scratch row so the append loop can index them, and one
    // append (two SADDR dword stores, the cursor advanced in place) per set bit,
    // the wave looping max-over-lanes(popcount) times — 1 or 2 late in a scan.
    auto max16 = [&](const f32x16& acc) {
        float m = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, acc[r]), acc[r + 1]);
        return fmaxf(m, acc[15]);
    };
    auto appends = [&](const f32x16& acc, int64_t sub0, float m) {
        if (__ballot(m >= thr) == 0) return;
        uint32_t bits = 0u;  // bit 15-r <=> acc[r] passes
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
        if (bits) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<float4*>(wscr + 4 * i) =
                    make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]);
        }
        const uint32_t sub_lane = static_cast<uint32_t>(sub0) + static_cast<uint32_t>(4 * half);
        while (__ballot(bits != 0u)) {
            issued += 2;  // exactly two store instructions for the wave
            if (bits) {
                const int b = 31 - __builtin_clz(bits);  // highest set bit = lowest r
                bits &= ~(1u << b);
                const int r = 15 - b;
                const float v = wscr[r];  // same-wave LDS write → read: in order
                const uint32_t id = sub_lane + static_cast<uint32_t>((r & 3) + 8 * (r >> 2));
                asm volatile(
                    "global_store_dword %0, %1, %2\n\tglobal_store_dword %0, %3, %2 offset:4\n\t"
                    "v_add_u32 %0, 8, %0"
                    : "+v"(woff)
                    : "v"(v), "s"(wbase), "v"(id)
                    : "memory");
            }
        }
    };
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
#pragma unroll
        for (int j = 0; j < kRing - 1; ++j) mk[j] = issued;  // drained
    };
    auto select = [&](const f32x16& acc, int64_t sub0) { appends(acc, sub0, max16(acc)); };

    // ---- scan ----
    // A fragment (row block rt, k step s) of the stage in buffer cur: the lane
    // reads item row rt*32 + col, bytes [32 s + 16 half, +16) — one VGPR base per
    // stage, the rest immediate offsets
    const int a_lane = col * C::RS + half * 16;
    auto lds_a = [&](frag (&af)[S], const char* stage, int rt) {
#pragma unroll
        for (int s = 0; s < S; ++s)
            af[s] = __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(stage + rt * 32 * C::RS + s * 32));
    };
    // one sub-tile: acc = its scores; prev (the sub-tile before, item base subp)
    // compared in the MFMA gaps, then appended
    // one sub-tile: acc = its scores; prev (the sub-tile before, item base subp)
    // max-reduced in the MFMA gaps, then filtered / appended
    auto step = [&](const frag (&af)[S], f32x16& acc, const f32x16& prev, int64_t subp) {
        acc = f32x16{};
        float m = 0.f;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            acc = M::run(af[s], qf[s], acc);
            if (s == 0) m = fmaxf(fmaxf(prev[0], prev[1]), prev[2]);
            if (s == 1) m = fmaxf(fmaxf(m, prev[3]), prev[4]);
            if (s == 2) m = fmaxf(fmaxf(m, prev[5]), prev[6]);
            if (s == 3) m = fmaxf(fmaxf(m, prev[7]), prev[8]);
            if (s == 4 || (S < 8 && s == S - 1)) {
                m = fmaxf(fmaxf(m, prev[9]), prev[10]);
                m = fmaxf(fmaxf(m, prev[11]), prev[12]);
                m = fmaxf(fmaxf(m, prev[13]), prev[14]);
                m = fmaxf(m, prev[15]);
            }
        }
        appends(prev, subp, m);
    };
    auto mask_tail = [&](f32x16& acc, int64_t sub0) {
        const int left = static_cast<int>(i_end - sub0);
        if (left < 32) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (tile_row(r, half) >= left) acc[r] = -INFINITY;
        }
    };

    // prologue: stages 0 .. kRing-2 in flight, stage 0 landed
    int mark0 = 0;
#pragma unroll
    for (int b = 0; b < kRing - 1; ++b) {
        if (i_begin + b * C::NT < i_end) fetch(i_begin + b * C::NT, b);
        if (b == 0) mark0 = issued;
        else mk[b - 1] = issued;
    }
    wait_vm_le(issued - mark0);
    raw_barrier();
    RT_PT(uint64_t pc_wait = 0, pc_bar = 0, pc_steps = 0, pc_cmp = 0; const uint64_t pc_start = clock64();)

    frag af[S];  // one set: sub-tile t+1's reads refill each fragment once t's MFMA on it has issued
    f32x16 accA, accB;
#pragma unroll
    for (int r = 0; r < 16; ++r) accB[r] = -INFINITY;  // "previous" of the first sub-tile: no passes
    int64_t subB = i_begin, subA = i_begin;
    bool last_in_a = false;
    int cur = 0;
    if (i_begin < i_end) lds_a(af, &tile[0][0] + a_lane, 0);
    for (int64_t t0 = i_begin; t0 < i_end; t0 += C::NT) {
        const bool more = t0 + C::NT < i_end;
        const int rem = static_cast<int>(i_end - t0 < C::NT ? i_end - t0 : C::NT);  // rows in this stage
        if (t0 + (kRing - 1) * C::NT < i_end) fetch(t0 + (kRing - 1) * C::NT, cur == 0 ? kRing - 1 : cur - 1);
        mk[kRing - 2] = issued;
        const char* stage = &tile[cur][0] + a_lane;
        RT_PT(const uint64_t c4s = clock64();)
#if !RT_TOPK3_PAIRCMP
        maybe_compact();  // the only call site in the loop (keeps the call's register saves out of the steps)
#endif
        RT_PT(const uint64_t c5s = clock64(); pc_cmp += c5s - c4s;)
        // sub-tiles in accumulators A, B, A, B, ... (the previous stage ended on B);
        // each sub-tile's A fragments are read while the one before computes
#if RT_TOPK3_PAIRCMP
#pragma unroll 1
#else
#pragma unroll
#endif
        for (int pr = 0; pr < C::NSUB / 2; ++pr) {
            const int r0 = 2 * pr, r1 = 2 * pr + 1;
#if RT_TOPK3_PAIRCMP
            maybe_compact();  // one call site: the pair loop is not unrolled
#endif
            if (r0 * 32 < rem) {
                step(af, accA, accB, subB);
                if (r1 * 32 < rem) lds_a(af, stage, r1);
                if (rem < (r0 + 1) * 32) mask_tail(accA, t0 + r0 * 32);
                subA = t0 + r0 * 32;
                last_in_a = true;
                if (r1 * 32 < rem) {
                    step(af, accB, accA, subA);
                    if (r1 + 1 < C::NSUB && (r1 + 1) * 32 < rem) lds_a(af, stage, r1 + 1);
                    if (rem < (r1 + 1) * 32) mask_tail(accB, t0 + r1 * 32);
                    subB = t0 + r1 * 32;
                    last_in_a = false;
                }
            }
        }
        RT_PT(const uint64_t c6 = clock64(); pc_steps += c6 - c5s;)
        if (more) wait_vm_le(issued - mk[0]);  // the next stage's DMA has landed
        RT_PT(const uint64_t c7 = clock64(); pc_wait += c7 - c6;)
        raw_barrier();
        RT_PT(pc_bar += clock64() - c7;)
#pragma unroll
        for (int j = 0; j + 1 < kRing - 1; ++j) mk[j] = mk[j + 1];
        cur = cur == kRing - 1 ? 0 : cur + 1;
        if (more) lds_a(af, &tile[cur][0] + a_lane, 0);
    }
    if (i_begin < i_end) {
        if (last_in_a) select(accA, subA);
        else select(accB, subB);
        maybe_compact();
    }

    RT_PT(const uint64_t c4 = clock64();)
    // ---- final selection, one query of the wave at a time (as v2) ----
    __threadfence_block();
    float* os = a.out_s + static_cast<int64_t>(split) * nq * k;
    int64_t* oi = a.out_i + static_cast<int64_t>(split) * nq * k;
    // one query of the wave at a time; a query whose buffer holds <= 128 entries
    // (the common case) is sorted from registers loaded while the previous query
    // sorted, so the global-load latency is paid once, not 32 times
    const int cnt_all = static_cast<int>((woff - woff0) / sizeof(Cand));
    auto load2 = [&](int c, float (&sv)[2], uint32_t (&iv)[2]) {
        const Cand* b = cbase + static_cast<int64_t>(c) * kCap;
        const int n0 = __shfl(cnt_all, c, 64), n1 = __shfl(cnt_all, c + 32, 64);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = lane * 2 + j;
            const Cand e = r < n0 + n1 ? v2::entry(b, n0, r) : Cand{-INFINITY, kEmptyId};
            sv[j] = e.s;
            iv[j] = e.i;
        }
    };
    float sn[2];
    uint32_t in[2];
    const int nvalid = static_cast<int>(nq - qw < 32 ? (nq - qw > 0 ? nq - qw : 0) : 32);
    if (nvalid > 0) load2(0, sn, in);
    for (int c = 0; c < nvalid; ++c) {
        const int64_t gq = qw + c;
        float sc[2] = {sn[0], sn[1]};
        uint32_t ic[2] = {in[0], in[1]};
        if (c + 1 < nvalid) load2(c + 1, sn, in);  // in flight during this query's sort
        int n0 = __shfl(cnt_all, c, 64), n1 = __shfl(cnt_all, c + 32, 64);
        float* orow = os + gq * k;
        int64_t* irow = oi + gq * k;
        if (n0 + n1 <= 128) {
            wave_sort_regs<2>(sc, ic);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = lane * 2 + j;
                if (r < k) {
                    const bool ok = ic[j] != kEmptyId;
                    orow[r] = ok ? sc[j] : -FLT_MAX;
                    irow[r] = ok ? static_cast<int64_t>(ic[j]) + a.id_offset : -1;
                }
            }
        } else {
            Cand* b = cbase + static_cast<int64_t>(c) * kCap;
            float nt;
            const int nn = compact_query(b, n0, n1, k, whist, nt);
            n0 = (nn + 1) >> 1;
            n1 = nn >> 1;
            if (n0 + n1 <= 128) emit_sorted<2>(b, n0, n1, k, orow, irow, a.id_offset);
            else emit_sorted<kE>(b, n0, n1, k, orow, irow, a.id_offset);
        }
    }
#ifdef RT_TOPK_PROBE_TIMING
    {
        const uint64_t c5 = clock64();
        const int64_t gw = static_cast<int64_t>(blockIdx.x) * kWavesB + wave;
        if (lane == 0 && gw < 65536) {
            uint64_t* o = probe_cycles + gw * 6;
            o[0] = c5 - pc_start; o[1] = pc_wait; o[2] = pc_bar; o[3] = pc_steps; o[4] = pc_cmp; o[5] = c5 - c4;
        }
    }
#endif
}

template <typename T, int S>
int launch_S(const Args& a, int splits, int64_t items_per_split, hipStream_t st) {
    const int64_t q_tiles = (a.nq + kQT - 1) / kQT;
    dim3 grid(static_cast<unsigned>(q_tiles * splits));
    if (a.excl)
        hipLaunchKernelGGL((flatip_topk_v3_kernel<T, S, true>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split);
    else
        hipLaunchKernelGGL((flatip_topk_v3_kernel<T, S, false>), grid, dim3(64 * kWavesB), 0, st, a, splits,
                           items_per_split);
    return check_launch("flatip_topk_v3_kernel");
}

}  // namespace v3
}  // namespace topk
}  // namespace rt
