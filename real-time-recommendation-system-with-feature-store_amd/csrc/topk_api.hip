// C ABI for the Flat-IP top-K (rt_flatip_topk) and the candidate-list merge
// (rt_topk_merge, used for split corpora and for the multi-GPU merge of
// per-shard top-K lists after an RCCL all-gather).
#include <array>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>

#include "topk_impl.h"

namespace rt {
namespace topk {

// ---- merge [n_lists][nq][k_in] → [nq][k_out], one wave per query ----
// Candidates stream through a per-wave LDS buffer of N entries: the first
// k_out slots keep the running best, the rest take new candidates, then sort.
// ids are carried as uint32 (0 <= id < 2^32-1).
constexpr int kMergeN = 1024;

// Small merges (n_lists·k_in <= 64·E, k_out <= 64·E; C3's 9 lists of 10, two
// shards of 100) sort in registers: E candidates per lane, one register
// bitonic sort, no LDS (the LDS form below costs ~16 µs at C3).
template <int E>
__global__ __launch_bounds__(256) void topk_merge_regs_kernel(const float* __restrict__ s_in,
                                                              const int64_t* __restrict__ i_in, int64_t nq,
                                                              int n_lists, int k_in, int k_out,
                                                              float* __restrict__ s_out,
                                                              int64_t* __restrict__ i_out) {
    const int lane = threadIdx.x & 63;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int total = n_lists * k_in;
    float sv[E];
    uint32_t iv[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int e = lane * E + j;
        sv[j] = -INFINITY;
        iv[j] = kEmptyId;
        if (e < total) {
            const int l = e / k_in, c = e - l * k_in;
            const int64_t off = (static_cast<int64_t>(l) * nq + q) * k_in + c;
            const int64_t id = i_in[off];
            if (id >= 0) { sv[j] = s_in[off]; iv[j] = static_cast<uint32_t>(id); }
        }
    }
    wave_sort_regs<E>(sv, iv);
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int e = lane * E + j;
        if (e < k_out) {
            const bool ok = iv[j] != kEmptyId;
            s_out[q * k_out + e] = ok ? sv[j] : -FLT_MAX;
            i_out[q * k_out + e] = ok ? static_cast<int64_t>(iv[j]) : -1;
        }
    }
}

__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ s_in,
                                                         const int64_t* __restrict__ i_in, int64_t nq,
                                                         int n_lists, int k_in, int k_out,
                                                         float* __restrict__ s_out,
                                                         int64_t* __restrict__ i_out) {
    __shared__ Cand buf[4][kMergeN];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (q >= nq) return;
    Cand* b = buf[w];
    const int64_t total = static_cast<int64_t>(n_lists) * k_in;
    int want = total < kMergeN ? static_cast<int>(total) : kMergeN;
    if (want < k_out + 64) want = k_out + 64;  // room for new candidates each round
    int n = next_pow2(want);
    if (n > kMergeN) n = kMergeN;
    int kept = 0;
    int64_t next = 0;
    for (;;) {
        for (int e = kept + lane; e < n; e += 64) {
            const int64_t src = next + (e - kept);
            Cand c{-INFINITY, kEmptyId};
            if (src < total) {
                const int l = static_cast<int>(src / k_in);
                const int j = static_cast<int>(src - static_cast<int64_t>(l) * k_in);
                const int64_t off = (static_cast<int64_t>(l) * nq + q) * k_in + j;
                const int64_t id = i_in[off];
                if (id >= 0) c = Cand{s_in[off], static_cast<uint32_t>(id)};
            }
            b[e] = c;
        }
        next += n - kept;
        wave_lds_sync();
        wave_sort_lds(b, n);
        kept = k_out;
        if (next >= total) break;
    }
    for (int e = lane; e < k_out; e += 64) {
        const Cand c = b[e];
        const bool ok = c.i != kEmptyId;
        s_out[q * k_out + e] = ok ? c.s : -FLT_MAX;
        i_out[q * k_out + e] = ok ? static_cast<int64_t>(c.i) : -1;
    }
}

// Merges of <= 1024 candidates into <= 128 (the owner merge of the multi-GPU
// top-K: N lists of k = 100; C3's split lists): the v4 finish's register
// select. Each lane holds 16 candidates as composite keys (score key << 32 |
// ~id), a radix select starting below the keys' shared prefix cuts them to
// <= 128, and the unrolled 128-entry sort writes the k_out best — instead of a
// 512/1024-entry LDS bitonic sort (176 us for 8 lists x 8,192 queries).
__global__ __launch_bounds__(256) void topk_merge_select_kernel(const float* __restrict__ s_in,
                                                                const int64_t* __restrict__ i_in, int64_t nq,
                                                                int n_lists, int k_in, int k_out,
                                                                float* __restrict__ s_out,
                                                                int64_t* __restrict__ i_out) {
    constexpr int R = v4::kFinishRegs;
    __shared__ __attribute__((aligned(16))) uint32_t hist_all[4][256];
    __shared__ __attribute__((aligned(16))) Cand keep_all[4][v4::kFinishCap];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (q >= nq) return;
    const int total = n_lists * k_in;  // <= 64 R (host-checked)
    uint64_t key[R];
    uint32_t vmask = 0u;
    // slot e of this lane: flat entry f = 64 e + lane = (list l, position j)
    int l = lane / k_in, j = lane - (lane / k_in) * k_in;
#pragma unroll
    for (int e = 0; e < R; ++e) {
        key[e] = 0ull;
        if (e * 64 + lane < total) {
            const int64_t off = (static_cast<int64_t>(l) * nq + q) * k_in + j;
            const int64_t id = i_in[off];
            if (id >= 0) {
                key[e] = v4::ckey(Cand{s_in[off], static_cast<uint32_t>(id)});
                vmask |= 1u << e;
            }
        }
        j += 64;
        while (j >= k_in) { j -= k_in; ++l; }
    }
    uint64_t mx = 0ull, mn = ~0ull;
    int nv = 0;
#pragma unroll
    for (int e = 0; e < R; ++e)
        if ((vmask >> e) & 1u) {
            mx = key[e] > mx ? key[e] : mx;
            mn = key[e] < mn ? key[e] : mn;
            ++nv;
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(mx, o, 64), b = __shfl_xor(mn, o, 64);
        mx = a > mx ? a : mx;
        mn = b < mn ? b : mn;
        nv += __shfl_xor(nv, o, 64);
    }
    Cand* keep = keep_all[w];
    int m = 0;
    if (nv > 0) {
        int shift = 64 - (mx == mn ? 64 : __builtin_clzll(mx ^ mn));  // bits below the shared prefix
        if (shift < 8) shift = 8;
        uint64_t prefix = mx & v4::prefix_mask(shift);
        int kept = nv;
        auto eachr = [&](auto&& fn) {
#pragma unroll
            for (int e = 0; e < R; ++e)
                if ((vmask >> e) & 1u) fn(key[e]);
        };
        if (nv > v4::kFinishCap) v4::radix_prefix(eachr, k_out, v4::kFinishCap, hist_all[w], prefix, shift, kept);
        const uint64_t pmask = v4::prefix_mask(shift);
        // entries above the boundary bucket first, then the bucket up to the
        // cap: a bucket still over the cap after all 64 bits holds copies of one
        // (score, id) — the same entry listed twice — so any of them may go
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int e = 0; e < R; ++e) {
                const uint64_t kb = key[e] & pmask;
                const bool take = ((vmask >> e) & 1u) && (pass == 0 ? kb > prefix : kb == prefix);
                const uint64_t bm = __ballot(take);
                const int pos = m + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                        static_cast<uint32_t>(bm >> 32),
                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bm), 0u)));
                if (take && pos < v4::kFinishCap)
                    keep[pos] = Cand{v2::okey_inv(static_cast<uint32_t>(key[e] >> 32)), ~static_cast<uint32_t>(key[e])};
                m += __popcll(bm);
            }
        }
        if (m > v4::kFinishCap) m = v4::kFinishCap;
    }
    wave_lds_sync();
    v4::finish_sort<2>(keep, m, k_out, s_out + q * k_out, i_out + q * k_out, 0);
}

int launch_merge(const float* s, const int64_t* ids, int64_t nq, int n_lists, int k_in, int k_out,
                 float* os, int64_t* oi, hipStream_t st) {
    if (k_out + 64 > kMergeN) return RT_ERR_UNSUPPORTED;
    dim3 grid(static_cast<unsigned>((nq + 3) / 4));
    const int64_t total = static_cast<int64_t>(n_lists) * k_in;
    if (total <= 64 * v4::kFinishRegs && k_out <= v4::kFinishCap)
        hipLaunchKernelGGL(topk_merge_select_kernel, grid, dim3(256), 0, st, s, ids, nq, n_lists, k_in, k_out, os, oi);
    else if (total <= 128 && k_out <= 128)
        hipLaunchKernelGGL(topk_merge_regs_kernel<2>, grid, dim3(256), 0, st, s, ids, nq, n_lists, k_in, k_out, os, oi);
    else if (total <= 256 && k_out <= 256)
        hipLaunchKernelGGL(topk_merge_regs_kernel<4>, grid, dim3(256), 0, st, s, ids, nq, n_lists, k_in, k_out, os, oi);
    else
        hipLaunchKernelGGL(topk_merge_kernel, grid, dim3(256), 0, st, s, ids, nq, n_lists, k_in, k_out, os, oi);
    return check_launch("topk_merge_kernel");
}

inline Shape shape_for(int dtype, int d, int k) {
    return dtype == RT_F32 ? shape_f32(d, k) : dtype == RT_F16 ? shape_f16(d, k) : shape_bf16(d, k);
}

constexpr int64_t kCUs = 256;  // MI355X compute units

// planner overrides for tests and tuning (rt_flatip_topk_tuning)
static int g_v4_mode = 0;     // 0 auto, 1 never, 2 wherever legal
static int g_v4_stride = 0;   // 0: planner's choice
static int g_v4_rank = -1;    // -1: planner's choice; 0: no sample (v2-style running threshold)
static int g_v4_joint = 1;    // 1: over several splits, one corpus-wide threshold per query
static int g_dense = 1;       // 1: fp32 small corpora take the GEMM + select pair (topk_dense.h)
static int g_v4_presample = 1;  // 1: joint thresholds from one sample-only launch over every split

// Smallest failure-safe rank: the least r in [1, r_max] with P(Bin(n, f) >= r)
// <= 1e-6 (r > n: probability 0, safe), 0 when none. The binomial tail of
// every r comes from one pass over the pmf (n <= kMaxK terms), summed from the
// top — the planner below evaluates it for up to 63 strides per plan, on the
// host path of every search call (a log-sum-exp tail per (stride, rank) pair
// cost ~1.7 ms per call at the C4 shapes).
inline int safe_rank(int n, double f, int r_max) {
    static const auto lf = [] {  // log i!
        std::array<double, kMaxK + 2> t{};
        for (int i = 0; i <= kMaxK + 1; ++i) t[i] = std::lgamma(i + 1.0);
        return t;
    }();
    if (n < 0 || n > kMaxK || !(f > 0.0)) return 0;
    if (f >= 1.0) return n + 1 <= r_max ? n + 1 : 0;  // X = n: only r > n is safe
    double tail[kMaxK + 2];
    tail[n + 1] = 0.0;
    const double lf_ = std::log(f), lg = std::log1p(-f);
    for (int i = n; i >= 0; --i) tail[i] = tail[i + 1] + std::exp(lf[n] - lf[i] - lf[n - i] + i * lf_ + (n - i) * lg);
    for (int r = 1; r <= r_max; ++r)
        if (r > n || tail[r] <= 1e-6) return r;
    return 0;
}

// the v4 sample: the sparsest stride whose smallest safe rank keeps the expected
// candidates per query, rank/f, within RT_TOPK_V4_APPEND_CAP. "Safe": the
// estimate overshoots the split's k-th score (a rescan) with probability <= 1e-6
// — P(>= rank of the split's top k fall in the sample) for a 1/f sample; the
// group-maximum estimate sits at or below the item rank, so this bounds it.
// Cap 500 (round 6; 960 before): k = 100 at the C4 shard and the 1M corpus
// takes stride 32 / rank 15 (~460 appends) instead of 64 / 11 (~670): the
// twice denser sample costs less than the appends and finish input it saves,
// 3-7 % at 125K and 2 % at 1M (profiles/r06_topk_stride_sweep.txt).
#ifndef RT_TOPK_V4_APPEND_CAP
#define RT_TOPK_V4_APPEND_CAP 500.0
#endif
#ifndef RT_TOPK_V4_MAX_STRIDE
#define RT_TOPK_V4_MAX_STRIDE 64
#endif
// (stride, rank) of the v4 sample over `items_per_split` rows: the largest
// stride whose failure-safe rank keeps the expected appends (rank * stride,
// per query) within RT_TOPK_V4_APPEND_CAP
inline void plan_v4_sample(int k, int64_t items_per_split, int& stride, int& rank) {
    const int64_t nst = (items_per_split + v4::Cfg4<__half, 8>::NT - 1) / v4::Cfg4<__half, 8>::NT;
    stride = 0;
    rank = 0;
    for (int st = RT_TOPK_V4_MAX_STRIDE; st >= 2; --st) {
        const int64_t nsa = (nst + st - 1) / st;
        if (nsa < 4) continue;  // fewer than 32 groups per query in the sample
        const double f = static_cast<double>(nsa) / static_cast<double>(nst);
        const int r = safe_rank(k, f, 2 * v4::kList);
        if (r > 0 && r / f <= RT_TOPK_V4_APPEND_CAP) { stride = st; rank = r; return; }
    }
}

// the same, for a sample taken split by split (every stride-th stage of each
// split: the presampled plan, or shards of a corpus on several GPUs): the
// sampled fraction is sum_s ceil(stages_s / stride) / stages
inline void plan_v4_sample_split(int k, int64_t nx, int64_t items_per_split, int& stride, int& rank) {
    constexpr int NT = v4::Cfg4<__half, 8>::NT;
    const int64_t nst = (nx + NT - 1) / NT;
    const int64_t sps = (items_per_split + NT - 1) / NT;  // stages per full split
    const int64_t nfull = nst / sps, rem = nst - nfull * sps;
    stride = 0;
    rank = 0;
    for (int st = RT_TOPK_V4_MAX_STRIDE; st >= 2; --st) {
        const int64_t nsa = nfull * ((sps + st - 1) / st) + (rem + st - 1) / st;
        if (nsa < 4) continue;
        const double f = static_cast<double>(nsa) / static_cast<double>(nst);
        const int r = safe_rank(k, f, 2 * v4::kList);
        if (r > 0 && r / f <= RT_TOPK_V4_APPEND_CAP) { stride = st; rank = r; return; }
    }
}

// (stride, rank) per (kind, k, rows, rows per split), computed once per shape
inline void plan_v4_sample_cached(bool split_form, int k, int64_t nx, int64_t items_per_split, int& stride,
                                  int& rank) {
    static std::mutex mu;
    static std::map<std::tuple<bool, int, int64_t, int64_t>, std::pair<int, int>> memo;
    const auto key = std::make_tuple(split_form, k, nx, items_per_split);
    {
        std::lock_guard<std::mutex> g(mu);
        const auto it = memo.find(key);
        if (it != memo.end()) {
            stride = it->second.first;
            rank = it->second.second;
            return;
        }
    }
    if (split_form) plan_v4_sample_split(k, nx, items_per_split, stride, rank);
    else plan_v4_sample(k, items_per_split, stride, rank);
    std::lock_guard<std::mutex> g(mu);
    if (memo.size() > 4096) memo.clear();
    memo[key] = {stride, rank};
}

// v4 (sampled-threshold scan + finish) for 16-bit, d <= 128, 32 < k <= 128 over
// a large corpus with enough queries to fill the chip at <= 8 item splits
inline bool plan_v4(int64_t nq, int64_t nx, int d, int dtype, int k, Plan& p) {
    if (g_v4_mode == 1) return false;
    if (dtype == RT_F32 || d > 128 || k > v4::kMaxK) return false;
    const bool forced = g_v4_mode == 2;
    if (!forced && (k <= v3::kMaxKv3 || nx < 65536)) return false;
    constexpr int QT = v4::Geo<v4::kQS>::QT;
    p.chunk = nq < kQueryChunk ? nq : kQueryChunk;
    if (p.chunk < 1) p.chunk = 1;
    p.q_tiles = static_cast<int>((p.chunk + QT - 1) / QT);
    // enough query tiles that <= kMaxSplits item splits fill the chip (the
    // 8,192-query slice of one of 8 GPUs: 16 tiles x 16 splits)
    if (!forced && static_cast<int64_t>(p.q_tiles) * v4::kMaxSplits < kCUs) return false;
    int splits = 1;
    while (splits < v4::kMaxSplits && static_cast<int64_t>(p.q_tiles) * splits < kCUs) splits *= 2;
    constexpr int NT = v4::Cfg4<__half, 8>::NT;
    int64_t tiles = (nx + NT - 1) / NT;
    while (splits > 1 && tiles / splits < 8) splits /= 2;
    int64_t tiles_per = (tiles + splits - 1) / splits;
    if (tiles_per < 1) tiles_per = 1;
    p.items_per_split = tiles_per * NT;
    p.splits = static_cast<int>(nx > 0 ? (nx + p.items_per_split - 1) / p.items_per_split : 1);
    p.cap = v4::kCap;
    p.v4 = 1;
    // several splits: one threshold per query from a sample of the whole corpus
    // (the union of the splits' buffers then holds ~rank*stride entries, not
    // splits times that); one split: the per-split form
    p.v4_joint = (p.splits > 1 && g_v4_joint) ? 1 : 0;
    p.v4_presample = (p.v4_joint && g_v4_presample) ? 1 : 0;
    if (p.v4_presample) plan_v4_sample_cached(true, k, nx, p.items_per_split, p.stride, p.rank);
    else plan_v4_sample_cached(false, k, 0, p.v4_joint ? nx : p.items_per_split, p.stride, p.rank);
    if (p.v4_presample && (p.stride <= 0 || p.rank <= 0)) p.v4_presample = 0;  // no sample fits: round-4 form
    if (g_v4_stride > 0) p.stride = g_v4_stride;
    if (g_v4_rank >= 0) p.rank = g_v4_rank;
    const int64_t q_pad = static_cast<int64_t>(p.q_tiles) * QT;
    p.cand_bytes = static_cast<size_t>(p.splits) * q_pad * v4::kCap * sizeof(Cand);
    p.meta_bytes = static_cast<size_t>(p.splits) * q_pad * 2 * sizeof(int);
    p.fail_bytes = p.v4_joint ? static_cast<size_t>(q_pad) * sizeof(int) : 0;
    p.lists_bytes = p.v4_presample ? static_cast<size_t>(p.splits) * q_pad * v4::kSampleList * sizeof(float) : 0;
    p.thr_bytes = p.v4_presample ? static_cast<size_t>(q_pad) * sizeof(float) : 0;
    p.part_bytes = 0;
    return true;
}

inline Plan make_plan(int64_t nq, int64_t nx, int d, int dtype, int k, const Shape& sh) {
    Plan p{};
    if (nx > 0 && plan_v4(nq, nx, d, dtype, k, p)) return p;
    if (dtype == RT_F32 && g_dense && dense::applies(nx, d, k)) {
        // the score slab of one query chunk (<= 256 MB: it stays in the Infinity Cache)
        p.dense = 1;
        p.chunk = dense::chunk_for(nq, nx);
        p.q_tiles = 1;
        p.splits = 1;
        p.items_per_split = nx;
        p.cand_bytes = static_cast<size_t>(p.chunk) * dense::ld_for(nx) * sizeof(float);
        return p;
    }
    p.chunk = nq < kQueryChunk ? nq : kQueryChunk;
    if (p.chunk < 1) p.chunk = 1;
    p.q_tiles = static_cast<int>((p.chunk + sh.qt - 1) / sh.qt);
    const int64_t tiles = (nx + sh.nt - 1) / sh.nt;
    int64_t splits;
    if (sh.kind == 2) {
        splits = v2::planned_splits(p.q_tiles, nx);
    } else {
        // at most 2 blocks per CU (<= 512 blocks: one co-resident wave of
        // blocks, no tail), >= 4 item tiles per split, <= 64 splits. C3 (48
        // query tiles x 54 item tiles): 9 splits = 432 blocks run 0.217 ms;
        // rounding up to 11 splits = 528 blocks (3 on some CUs) ran 0.244 ms,
        // 14 splits = 672 blocks 0.243 ms.
        splits = 2 * kCUs / p.q_tiles;
        int64_t max_splits = tiles / 4;
        if (max_splits < 1) max_splits = 1;
        if (splits > max_splits) splits = max_splits;
        if (splits > 64) splits = 64;
        if (splits < 1) splits = 1;
    }
    int64_t tiles_per = (tiles + splits - 1) / splits;
    if (tiles_per < 1) tiles_per = 1;
    p.items_per_split = tiles_per * sh.nt;
    p.splits = static_cast<int>(nx > 0 ? (nx + p.items_per_split - 1) / p.items_per_split : 1);
    p.cap = sh.cap;
    p.kth_bytes = (sh.kind == 0 && p.splits > 1) ? static_cast<size_t>(p.chunk) * sizeof(uint32_t) : 0;
    p.cand_bytes = static_cast<size_t>(p.splits) * p.q_tiles * sh.qt * p.cap * sizeof(Cand);
    p.part_bytes = p.splits > 1 ? static_cast<size_t>(p.splits) * p.chunk * k * (sizeof(float) + sizeof(int64_t)) : 0;
    return p;
}

inline size_t align256(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace topk
}  // namespace rt

using namespace rt;

extern "C" size_t rt_flatip_topk_workspace_bytes(int64_t nq, int64_t nx, int d, int dtype, int k) {
    if (nq <= 0 || k <= 0 || k > topk::kMaxK || d <= 0) return 256;
    if (dtype != RT_F32 && dtype != RT_F16 && dtype != RT_BF16) return 256;
    const topk::Plan p = topk::make_plan(nq, nx, d, dtype, k, topk::shape_for(dtype, d, k));
    return topk::align256(p.cand_bytes) + p.part_bytes + topk::align256(p.meta_bytes) + topk::align256(p.kth_bytes) +
           topk::align256(p.fail_bytes) + topk::align256(p.lists_bytes) + topk::align256(p.thr_bytes) + 256;
}

extern "C" int rt_flatip_topk(const void* queries, int64_t nq, const void* items, int64_t nx, int d,
                              int dtype, int k, const uint32_t* exclude_bits, int64_t exclude_words,
                              int64_t id_offset, float* out_scores, int64_t* out_ids, void* workspace,
                              size_t workspace_bytes, void* stream) {
    if (nq < 0 || nx < 0 || d <= 0 || k <= 0) return RT_ERR_INVALID;
    if (nq == 0) return RT_OK;
    if (!queries || !out_scores || !out_ids || (nx > 0 && !items)) return RT_ERR_INVALID;
    if (k > topk::kMaxK) return RT_ERR_UNSUPPORTED;
    if (dtype != RT_F32 && dtype != RT_F16 && dtype != RT_BF16) return RT_ERR_INVALID;
    if (dtype == RT_F32 ? (d % 4 != 0 || d > 256) : (d % 8 != 0 || d > 256)) return RT_ERR_UNSUPPORTED;
    if (nx >= 0xFFFFFFFFll || (id_offset + nx) >= 0xFFFFFFFFll || id_offset < 0) return RT_ERR_UNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(queries) | reinterpret_cast<uintptr_t>(items)) & 15) return RT_ERR_INVALID;
    if (exclude_bits && exclude_words < (nx + 31) / 32) return RT_ERR_INVALID;
    const topk::Plan p = topk::make_plan(nq, nx, d, dtype, k, topk::shape_for(dtype, d, k));
    const size_t cand_al = topk::align256(p.cand_bytes);
    if (!workspace ||
        workspace_bytes < cand_al + p.part_bytes + topk::align256(p.meta_bytes) + topk::align256(p.kth_bytes) +
                              topk::align256(p.fail_bytes) + topk::align256(p.lists_bytes) + topk::align256(p.thr_bytes))
        return RT_ERR_WORKSPACE;
    hipStream_t st = as_stream(stream);
    char* part = reinterpret_cast<char*>(workspace) + cand_al;
    int* meta = reinterpret_cast<int*>(part + p.part_bytes);
    uint32_t* kth = reinterpret_cast<uint32_t*>(part + p.part_bytes + topk::align256(p.meta_bytes));
    int* fail = reinterpret_cast<int*>(part + p.part_bytes + topk::align256(p.meta_bytes) + topk::align256(p.kth_bytes));
    float* v4_lists = reinterpret_cast<float*>(reinterpret_cast<char*>(fail) + topk::align256(p.fail_bytes));
    float* v4_thr = reinterpret_cast<float*>(reinterpret_cast<char*>(v4_lists) + topk::align256(p.lists_bytes));
    const size_t esz = dtype == RT_F32 ? 4 : 2;
    for (int64_t q0 = 0; q0 < nq; q0 += p.chunk) {
        const int64_t nc = (nq - q0) < p.chunk ? (nq - q0) : p.chunk;
        float* os = out_scores + q0 * k;
        int64_t* oi = out_ids + q0 * k;
        int rc;
        if (nx == 0) {  // empty corpus: every slot (-FLT_MAX, -1)
            rc = topk::launch_merge(os, oi, nc, 0, 1, k, os, oi, st);
            if (rc) return rc;
            continue;
        }
        topk::Args a{};
        a.Q = reinterpret_cast<const char*>(queries) + q0 * d * esz;
        a.nq = nc;
        a.X = items;
        a.nx = nx;
        a.d = d;
        a.k = k;
        a.excl = exclude_bits ? exclude_bits + q0 * exclude_words : nullptr;
        a.excl_words = exclude_words;
        a.cand = reinterpret_cast<Cand*>(workspace);
        a.id_offset = id_offset;
        a.meta = meta;
        a.fail = fail;
        a.v4_lists = v4_lists;
        a.v4_thr = v4_thr;
        if (p.kth_bytes) {
            a.kth_shared = kth;
            const hipError_t e = hipMemsetAsync(kth, 0, static_cast<size_t>(nc) * sizeof(uint32_t), st);
            if (e != hipSuccess) {
                set_last_error("hipMemsetAsync(topk kth)", e);
                return RT_ERR_HIP;
            }
        }
        if (p.splits > 1 && !p.v4) {  // per-split lists [split][nc][k], merged below
            a.out_s = reinterpret_cast<float*>(part);
            a.out_i = reinterpret_cast<int64_t*>(part + static_cast<size_t>(p.splits) * p.chunk * k * sizeof(float));
        } else {
            a.out_s = os;
            a.out_i = oi;
        }
        switch (dtype) {
            case RT_F32: rc = topk::launch_f32(a, p, st); break;
            case RT_F16: rc = topk::launch_f16(a, p, st); break;
            default: rc = topk::launch_bf16(a, p, st); break;
        }
        if (rc) return rc;
        if (p.splits > 1 && !p.v4) {
            rc = topk::launch_merge(a.out_s, a.out_i, nc, p.splits, k, k, os, oi, st);
            if (rc) return rc;
        }
    }
    return RT_OK;
}

// ---- corpus-sharded search with one corpus-wide threshold per query ----
// (several GPUs, each holding a row shard: rtrec_amd/dist/sharded.py::
// sharded_topk_global). Only where rt_flatip_topk plans the v4 kernel pair.
namespace rt {
namespace topk {
struct ShardArgs {
    Plan p;
    Args a;
    size_t need;
};
inline int shard_setup(const void* queries, int64_t nq, const void* items, int64_t nx, int d, int dtype, int k,
                       void* workspace, size_t workspace_bytes, ShardArgs& s) {
    if (nq <= 0 || nx <= 0 || d <= 0 || k <= 0 || k > v4::kMaxK) return RT_ERR_INVALID;
    if (dtype != RT_F16 && dtype != RT_BF16) return RT_ERR_UNSUPPORTED;
    if (d % 8 != 0 || d > 128) return RT_ERR_UNSUPPORTED;
    if (!queries || !items) return RT_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(queries) | reinterpret_cast<uintptr_t>(items)) & 15) return RT_ERR_INVALID;
    if (nx >= 0xFFFFFFFFll) return RT_ERR_UNSUPPORTED;
    s.p = make_plan(nq, nx, d, dtype, k, shape_for(dtype, d, k));
    if (!s.p.v4 || s.p.chunk < nq) return RT_ERR_UNSUPPORTED;  // one query chunk, the v4 plan
    const int64_t q_pad = static_cast<int64_t>(s.p.q_tiles) * v4::Geo<v4::kQS>::QT;
    const size_t lists = static_cast<size_t>(s.p.splits) * q_pad * v4::kSampleList * sizeof(float);
    s.need = align256(s.p.cand_bytes) + align256(s.p.meta_bytes) + align256(lists) + align256(q_pad * sizeof(float));
    if (!workspace || workspace_bytes < s.need) return RT_ERR_WORKSPACE;
    char* w = reinterpret_cast<char*>(workspace);
    s.a = Args{};
    s.a.Q = queries;
    s.a.nq = nq;
    s.a.X = items;
    s.a.nx = nx;
    s.a.d = d;
    s.a.k = k;
    s.a.cand = reinterpret_cast<Cand*>(w);
    s.a.meta = reinterpret_cast<int*>(w + align256(s.p.cand_bytes));
    s.a.v4_lists = reinterpret_cast<float*>(w + align256(s.p.cand_bytes) + align256(s.p.meta_bytes));
    return RT_OK;
}
inline int v4_scan(int dtype, const Args& a, const Plan& p, int stride, int rank, int mode, hipStream_t st) {
    return dtype == RT_F16 ? v4_scan_f16(a, p, stride, rank, mode, st) : v4_scan_bf16(a, p, stride, rank, mode, st);
}
}  // namespace topk
}  // namespace rt

extern "C" size_t rt_flatip_topk_shard_workspace_bytes(int64_t nq, int64_t nx, int d, int dtype, int k) {
    topk::ShardArgs s{};
    const int rc = topk::shard_setup(reinterpret_cast<const void*>(16), nq, reinterpret_cast<const void*>(16), nx, d,
                                     dtype, k, reinterpret_cast<void*>(16), ~size_t(0), s);
    return rc ? 0 : s.need + 256;
}

namespace rt {
namespace topk {
// {sampled stages, stages} of a shard under plan p: every split samples its
// stages 0, stride, 2·stride, ... (the mode-3 scan of v4_scan)
inline void shard_stage_counts(const Plan& p, int64_t nx, int stride, int64_t* counts) {
    constexpr int NT = v4::Cfg4<__half, 8>::NT;
    const int64_t nst = (nx + NT - 1) / NT, sps = (p.items_per_split + NT - 1) / NT;
    const int64_t nfull = nst / sps, rem = nst - nfull * sps;
    counts[0] = nfull * ((sps + stride - 1) / stride) + (rem + stride - 1) / stride;
    counts[1] = nst;
}
}  // namespace topk
}  // namespace rt

extern "C" int rt_flatip_topk_shard_plan(int64_t nq, int64_t nx, int d, int dtype, int k, int stride,
                                         int64_t* stage_counts) {
    if (stride < 1 || !stage_counts) return RT_ERR_INVALID;
    topk::ShardArgs s{};
    const int rc = topk::shard_setup(reinterpret_cast<const void*>(16), nq, reinterpret_cast<const void*>(16), nx, d,
                                     dtype, k, reinterpret_cast<void*>(16), ~size_t(0), s);
    if (rc) return rc;
    topk::shard_stage_counts(s.p, nx, stride, stage_counts);
    return RT_OK;
}

extern "C" int rt_flatip_topk_shard_sample(const void* queries, int64_t nq, const void* items, int64_t nx, int d,
                                           int dtype, int k, int stride, float* top32, int64_t* stage_counts,
                                           void* workspace, size_t workspace_bytes, void* stream) {
    topk::ShardArgs s{};
    int rc = topk::shard_setup(queries, nq, items, nx, d, dtype, k, workspace, workspace_bytes, s);
    if (rc) return rc;
    if (stride < 1 || !top32 || !stage_counts) return RT_ERR_INVALID;
    topk::shard_stage_counts(s.p, nx, stride, stage_counts);
    hipStream_t st = as_stream(stream);
    topk::Args b = s.a;
    b.lists_out = s.a.v4_lists;
    const int64_t q_pad = static_cast<int64_t>(s.p.q_tiles) * topk::v4::Geo<topk::v4::kQS>::QT;
    rc = topk::v4_scan(dtype, b, s.p, stride, 1, 3, st);
    if (rc) return rc;
    return topk::v4::launch_threshold(s.a.v4_lists, s.p.splits, q_pad * topk::v4::kSampleList, nq, 1, nullptr, top32,
                                      st);
}

extern "C" int rt_topk_sample_rank(int k, int64_t sampled_stages, int64_t stages, int* rank) {
    if (k <= 0 || k > topk::v4::kMaxK || sampled_stages <= 0 || stages < sampled_stages || !rank) return RT_ERR_INVALID;
    const double f = static_cast<double>(sampled_stages) / static_cast<double>(stages);
    // 0: no failure-safe rank within the lists (the caller scans from -inf)
    *rank = topk::safe_rank(k, f, topk::v4::kSampleList);
    return RT_OK;
}

extern "C" int rt_topk_sample_threshold(const float* lists, int n_lists, int64_t nq, int rank, float* thr,
                                        void* stream) {
    if (!lists || !thr || n_lists <= 0 || nq < 0 || rank < 1 || rank > topk::v4::kSampleList) return RT_ERR_INVALID;
    if (nq == 0) return RT_OK;
    return topk::v4::launch_threshold(lists, n_lists, nq * topk::v4::kSampleList, nq, rank, thr, nullptr,
                                      as_stream(stream));
}

extern "C" int rt_flatip_topk_shard_search(const void* queries, int64_t nq, const void* items, int64_t nx, int d,
                                           int dtype, int k, const float* thr, int64_t id_offset, float* out_scores,
                                           int64_t* out_ids, void* workspace, size_t workspace_bytes, void* stream) {
    topk::ShardArgs s{};
    int rc = topk::shard_setup(queries, nq, items, nx, d, dtype, k, workspace, workspace_bytes, s);
    if (rc) return rc;
    if (!thr || !out_scores || !out_ids || id_offset < 0 || (id_offset + nx) >= 0xFFFFFFFFll) return RT_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    topk::Args b = s.a;
    b.thr_in = thr;
    b.out_s = out_scores;
    b.out_i = out_ids;
    b.id_offset = id_offset;
    const int64_t q_pad = static_cast<int64_t>(s.p.q_tiles) * topk::v4::Geo<topk::v4::kQS>::QT;
    rc = topk::v4_scan(dtype, b, s.p, 0, 0, 4, st);
    if (rc) return rc;
    return topk::v4::launch_finish(b, s.p.splits, q_pad, 3, nullptr, st);  // no union check: a shard may hold < k
}

extern "C" int rt_flatip_topk_tuning(int v4_mode, int v4_stride, int v4_rank) {
    if (v4_mode < 0 || (v4_mode & 3) > 2 || v4_mode > 30 || v4_stride < 0 || v4_rank < -1 ||
        v4_rank > 2 * topk::v4::kList)
        return RT_ERR_INVALID;
    topk::g_v4_presample = (v4_mode & 16) ? 0 : 1;
    v4_mode &= 15;
    topk::g_dense = (v4_mode & 8) ? 0 : 1;
    v4_mode &= 7;
    topk::g_v4_joint = (v4_mode & 4) ? 0 : 1;
    v4_mode &= 3;
    topk::g_v4_mode = v4_mode;
    topk::g_v4_stride = v4_stride;
    topk::g_v4_rank = v4_rank;
    return RT_OK;
}

extern "C" int rt_topk_merge(const float* scores, const int64_t* ids, int64_t nq, int n_lists, int k_in,
                             int k_out, float* out_scores, int64_t* out_ids, void* stream) {
    if (nq < 0 || n_lists < 0 || k_in <= 0 || k_out <= 0) return RT_ERR_INVALID;
    if (nq == 0) return RT_OK;
    if (!out_scores || !out_ids || (n_lists > 0 && (!scores || !ids))) return RT_ERR_INVALID;
    if (k_out > topk::kMaxK) return RT_ERR_UNSUPPORTED;
    return topk::launch_merge(scores, ids, nq, n_lists, k_in, k_out, out_scores, out_ids, as_stream(stream));
}
