// Offline-evaluation kernels: the train-item exclusion
// bitmap of generate_recommendations (scripts/evaluate_model.py:220-228) and
// the ranking metrics of Evaluator.evaluate (src/evaluation/metrics.py:73-228,
// 248-319) — Recall / Precision / NDCG / HitRate @k, reciprocal rank, average
// precision, coverage — computed per query row on the device.
//
// Integer / index work, HBM/latency-bound: one wave per query row, ranks by
// ballot + popcount, set membership by binary search in sorted CSR segments.
// Per-row metric terms are accumulated in the reference's order (rank
// ascending, fp64) by a wave-uniform walk over the hit bits, so the values
// follow the reference's sequential float64 sums.
#include "rt_common.h"

namespace rt {
namespace evalm {

constexpr int kMaxK = RT_METRICS_MAX_K;

struct KList {
    int v[kMaxK];
    int n;
};

__device__ __forceinline__ bool seg_contains(const int32_t* __restrict__ a, int64_t lo, int64_t hi, int64_t v) {
    if (v < INT32_MIN || v > INT32_MAX) return false;
    const int32_t x = static_cast<int32_t>(v);
    int64_t end = hi;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo < end && a[lo] == x;
}

// bits[r][w] = OR of (1 << (i - 32w)) over items i of CSR row (rows ? rows[r] : r)
// with 32w <= i < 32w + 32 and i < n_items; every word written (no pre-zeroing)
__global__ __launch_bounds__(256) void exclusion_bitmap_kernel(const int64_t* __restrict__ offsets,
                                                               const int32_t* __restrict__ items,
                                                               const int64_t* __restrict__ rows, int64_t n_csr_rows,
                                                               int64_t n_rows, int64_t n_items,
                                                               uint32_t* __restrict__ bits, int64_t words) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= n_rows * words) return;
    const int64_t r = t / words, w = t - r * words;
    const int64_t u = rows ? rows[r] : r;
    uint32_t word = 0u;
    if (u >= 0 && u < n_csr_rows) {
        int64_t lo = offsets[u], hi = offsets[u + 1];
        const int64_t first = 32 * w;
        // lower bound of `first` in the sorted segment
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (static_cast<int64_t>(items[mid]) < first) lo = mid + 1; else hi = mid;
        }
        for (int64_t i = lo; i < offsets[u + 1]; ++i) {
            const int64_t it = items[i];
            if (it >= first + 32 || it >= n_items) break;
            word |= 1u << static_cast<uint32_t>(it - first);
        }
    }
    bits[t] = word;
}

// One wave per query row r (columns of per_row: recall@k…, precision@k…,
// ndcg@k…, hit@k… for every k, then reciprocal rank, average precision).
__global__ __launch_bounds__(256) void rank_metrics_kernel(
    const int64_t* __restrict__ preds, int64_t n_rows, int list_len,
    const int64_t* __restrict__ gt_off, const int32_t* __restrict__ gt_items, const int64_t* __restrict__ gt_rows,
    int64_t n_gt_rows, const int64_t* __restrict__ ex_off, const int32_t* __restrict__ ex_items,
    const int64_t* __restrict__ ex_rows, int64_t n_ex_rows, KList K, int64_t num_items,
    double* __restrict__ per_row, int32_t* __restrict__ valid, uint32_t* __restrict__ cov) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n_rows) return;  // wave-uniform, no barriers below
    const int nk = K.n;
    const int ncols = 4 * nk + 2;
    double* out = per_row + r * ncols;
    const int64_t g = gt_rows ? gt_rows[r] : r;
    int64_t glo = 0, ghi = 0;
    if (g >= 0 && g < n_gt_rows) { glo = gt_off[g]; ghi = gt_off[g + 1]; }
    const int64_t n_gt = ghi - glo;
    if (n_gt <= 0) {  // Evaluator.evaluate skips users without ground truth
        for (int c = lane; c < ncols; c += 64) out[c] = 0.0;
        if (lane == 0) valid[r] = 0;
        return;
    }
    int64_t elo = 0, ehi = 0;
    if (ex_off) {
        const int64_t e = ex_rows ? ex_rows[r] : r;
        if (e >= 0 && e < n_ex_rows) { elo = ex_off[e]; ehi = ex_off[e + 1]; }
    }
    const int max_k = K.v[nk - 1];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes below this one
    int cnt[kMaxK];
    double dcg[kMaxK];
#pragma unroll
    for (int i = 0; i < kMaxK; ++i) { cnt[i] = 0; dcg[i] = 0.0; }
    double ap = 0.0;
    int first = -1, kept = 0, hits = 0;
    const int64_t* row = preds + r * static_cast<int64_t>(list_len);
    for (int j0 = 0; j0 < list_len; j0 += 64) {
        const int j = j0 + lane;
        const int64_t id = j < list_len ? row[j] : -1;
        const bool present = id >= 0;  // -1 pads a ragged prediction list
        const bool excl = present && elo < ehi && seg_contains(ex_items, elo, ehi, id);
        const bool keep = present && !excl;  // metrics.py:279-281: excluded items leave the list
        const uint64_t km = __ballot(keep);
        const int rank = kept + __popcll(km & lt);
        kept += __popcll(km);
        const bool hit = keep && seg_contains(gt_items, glo, ghi, id);
        if (cov && keep && rank < max_k && id < num_items) atomicOr(&cov[id >> 5], 1u << (id & 31));
        // the reference's loops, rank ascending (wave-uniform walk over the hit bits)
        uint64_t hm = __ballot(hit);
        while (hm) {
            const int src = __ffsll(static_cast<unsigned long long>(hm)) - 1;
            hm &= hm - 1;
            const int rk = __shfl(rank, src, 64);
            ++hits;
            if (first < 0) first = rk;
            ap += static_cast<double>(hits) / static_cast<double>(rk + 1);
#pragma unroll
            for (int i = 0; i < kMaxK; ++i) {
                if (i < nk && rk < K.v[i]) {
                    ++cnt[i];
                    dcg[i] += 1.0 / log2(static_cast<double>(rk) + 2.0);
                }
            }
        }
    }
    if (lane == 0) {
        for (int i = 0; i < nk; ++i) {
            const int k = K.v[i];
            out[i] = static_cast<double>(cnt[i]) / static_cast<double>(n_gt);
            out[nk + i] = static_cast<double>(cnt[i]) / static_cast<double>(k);
            const int64_t ideal = n_gt < k ? n_gt : k;
            double idcg = 0.0;
            for (int64_t q = 0; q < ideal; ++q) idcg += 1.0 / log2(static_cast<double>(q) + 2.0);
            out[2 * nk + i] = idcg > 0.0 ? dcg[i] / idcg : 0.0;
            out[3 * nk + i] = cnt[i] > 0 ? 1.0 : 0.0;
        }
        out[4 * nk] = first >= 0 ? 1.0 / static_cast<double>(first + 1) : 0.0;
        out[4 * nk + 1] = ap / static_cast<double>(n_gt);
        valid[r] = 1;
    }
}

// Column means over the valid rows, in a fixed order (deterministic): thread t
// sums rows t, t+256, … sequentially, then a fixed LDS tree; plus the number of
// valid rows and the coverage fraction popcount(cov) / num_items.
__global__ __launch_bounds__(256) void metrics_reduce_kernel(const double* __restrict__ per_row,
                                                             const int32_t* __restrict__ valid, int64_t n_rows,
                                                             int ncols, const uint32_t* __restrict__ cov,
                                                             int64_t num_items, double* __restrict__ out) {
    __shared__ double red[256];
    const int t = threadIdx.x;
    int64_t nv = 0;
    for (int64_t r = t; r < n_rows; r += 256) nv += valid[r] ? 1 : 0;
    red[t] = static_cast<double>(nv);
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s) red[t] += red[t + s];
        __syncthreads();
    }
    const double n_valid = red[0];
    __syncthreads();
    for (int c = 0; c < ncols; ++c) {
        double acc = 0.0;
        for (int64_t r = t; r < n_rows; r += 256)
            if (valid[r]) acc += per_row[r * ncols + c];
        red[t] = acc;
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if (t < s) red[t] += red[t + s];
            __syncthreads();
        }
        if (t == 0) out[c] = n_valid > 0.0 ? red[0] / n_valid : 0.0;
        __syncthreads();
    }
    int64_t pc = 0;
    if (cov && num_items > 0) {
        const int64_t words = (num_items + 31) / 32;
        for (int64_t w = t; w < words; w += 256) pc += __popc(cov[w]);
    }
    red[t] = static_cast<double>(pc);
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s) red[t] += red[t + s];
        __syncthreads();
    }
    if (t == 0) {
        out[ncols] = n_valid;
        out[ncols + 1] = (cov && num_items > 0) ? red[0] / static_cast<double>(num_items) : 0.0;
    }
}

}  // namespace evalm
}  // namespace rt

using namespace rt;

extern "C" int rt_exclusion_bitmap(const int64_t* offsets, const int32_t* items, int64_t n_csr_rows,
                                   const int64_t* rows, int64_t n_rows, int64_t n_items, uint32_t* bits,
                                   int64_t words, void* stream) {
    if (n_rows < 0 || n_items < 0 || n_csr_rows < 0 || words < (n_items + 31) / 32) return RT_ERR_INVALID;
    if (n_rows == 0 || words == 0) return RT_OK;
    if (!offsets || !bits) return RT_ERR_INVALID;  // items may be NULL when every segment is empty
    const int64_t total = n_rows * words;
    const int64_t blocks = (total + 255) / 256;
    if (blocks > (1ll << 31) - 1) return RT_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(evalm::exclusion_bitmap_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       as_stream(stream), offsets, items, rows, n_csr_rows, n_rows, n_items, bits, words);
    return check_launch("exclusion_bitmap_kernel");
}

extern "C" int rt_rank_metrics(const int64_t* preds, int64_t n_rows, int list_len, const int64_t* gt_offsets,
                               const int32_t* gt_items, const int64_t* gt_rows, int64_t n_gt_rows,
                               const int64_t* ex_offsets, const int32_t* ex_items, const int64_t* ex_rows,
                               int64_t n_ex_rows, const int32_t* k_values, int n_k, int64_t num_items,
                               double* per_row, int32_t* valid, uint32_t* coverage_bits, void* stream) {
    if (n_rows < 0 || list_len < 0 || n_k < 1 || n_k > evalm::kMaxK || !k_values) return RT_ERR_INVALID;
    evalm::KList K{};
    K.n = n_k;
    for (int i = 0; i < n_k; ++i) {  // host array, ascending positive
        if (k_values[i] <= 0 || (i > 0 && k_values[i] <= k_values[i - 1])) return RT_ERR_INVALID;
        K.v[i] = k_values[i];
    }
    if (n_rows == 0) return RT_OK;
    // item arrays may be NULL when every CSR segment is empty (offsets all 0)
    if (!per_row || !valid || !gt_offsets || (list_len > 0 && !preds)) return RT_ERR_INVALID;
    if (coverage_bits && num_items <= 0) return RT_ERR_INVALID;
    const int64_t blocks = (n_rows + 3) / 4;
    if (blocks > (1ll << 31) - 1) return RT_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(evalm::rank_metrics_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       as_stream(stream), preds, n_rows, list_len, gt_offsets, gt_items, gt_rows, n_gt_rows,
                       ex_offsets, ex_items, ex_rows, n_ex_rows, K, num_items, per_row, valid, coverage_bits);
    return check_launch("rank_metrics_kernel");
}

extern "C" int rt_rank_metrics_reduce(const double* per_row, const int32_t* valid, int64_t n_rows, int n_cols,
                                      const uint32_t* coverage_bits, int64_t num_items, double* out,
                                      void* stream) {
    if (n_rows < 0 || n_cols < 1 || !out || (n_rows > 0 && (!per_row || !valid))) return RT_ERR_INVALID;
    hipLaunchKernelGGL(evalm::metrics_reduce_kernel, dim3(1), dim3(256), 0, as_stream(stream), per_row, valid,
                       n_rows, n_cols, coverage_bits, num_items, out);
    return check_launch("metrics_reduce_kernel");
}
