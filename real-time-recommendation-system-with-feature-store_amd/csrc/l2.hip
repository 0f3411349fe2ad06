// IndexFlatL2 mode of the Flat index (FaissIndex with metric != "cosine",
// src/serving/retrieval.py:96-100): exact squared-L2 k-nearest neighbours on
// the same MFMA top-K kernels as the inner-product path.
//
// Ranking ‖q − x‖² ascending equals ranking q·x − ½‖x‖² descending, so both
// sides are AUGMENTED once (rt_l2_augment_f32): item rows [x, −½‖x‖², 0, 0, 0],
// query rows [q, 1, 0, 0, 0] (d + 4 columns, 16-byte rows; ‖x‖² a sequential
// fmaf chain, the oracle's order), and rt_flatip_topk selects k_sel >= k
// candidates on the augmented inner product. rt_l2_finish_f32 then recomputes
// the reported distance of every candidate exactly as Faiss's BLAS path
// defines it (exhaustive_L2sqr_blas: ‖q‖² + ‖x‖² − 2·q·x, clamped at 0; norms
// and the dot as sequential fmaf chains, the order oracle/flatip.c uses),
// re-sorts by (distance asc, id asc) — Faiss's max-heap keeps the lower id on
// exact ties — and keeps the k best. The augmented score and the reported
// distance round differently, so items can swap order near the k-th distance;
// the k_sel − k extra candidates (32 in kernels.flatl2_topk) absorb that, and
// the finish CERTIFIES each query: with the selection scores passed in, a
// query is flagged (unverified[q] = 1) unless the k-th reported distance sits
// below ‖q‖² − 2·s_last (s_last = the k_sel-th selection score, the best any
// unselected item can have) by more than a rounding bound of both quantities;
// the host re-selects flagged queries with a wider k_sel. Unfilled slots:
// (FLT_MAX, −1).
#include <float.h>

#include "rt_common.h"
#include "rt_sort.h"

namespace rt {
namespace l2 {

// one wave per row: copy the d columns, the augmented column and the zero pad
__global__ __launch_bounds__(256) void augment_kernel(const float* __restrict__ x, int64_t n, int d,
                                                      float* __restrict__ out, int ld_out, int role) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    const float* xr = x + r * d;
    float* o = out + r * ld_out;
    for (int c = lane; c < d; c += 64) o[c] = xr[c];
    float ss = 0.f;  // ||x||^2 in the finish pass's (and the oracle's) sequential order
    if (role == 1 && lane == 0)
        for (int c = 0; c < d; ++c) ss = __builtin_fmaf(xr[c], xr[c], ss);
    ss = __shfl(ss, 0, 64);
    for (int c = d + lane; c < ld_out; c += 64) o[c] = (c == d) ? (role == 0 ? 1.f : -0.5f * ss) : 0.f;
}

__device__ __forceinline__ float seq_dot(const float* __restrict__ a, const float* __restrict__ b, int d) {
    float acc = 0.f;
    for (int j = 0; j < d; ++j) acc = __builtin_fmaf(a[j], b[j], acc);
    return acc;
}

constexpr int kFinishN = 512;  // entries per wave (k <= 512)

// one wave per query: exact distances of the k_sel candidates, re-sorted, k kept
__global__ __launch_bounds__(256) void finish_kernel(const float* __restrict__ q_aug, int ld_q,
                                                     const float* __restrict__ x_aug, int ld_x, int d, int64_t nq,
                                                     int k_sel, const int64_t* __restrict__ sel_ids,
                                                     const float* __restrict__ sel_scores, int k,
                                                     float* __restrict__ scores, int64_t* __restrict__ ids,
                                                     int32_t* __restrict__ unverified, int64_t id_offset) {
    __shared__ Cand buf[4][kFinishN];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (q >= nq) return;  // wave-uniform; only wave-level LDS sync below
    const float* qr = q_aug + q * ld_q;
    const float qn = seq_dot(qr, qr, d);
    const int n = next_pow2(k_sel < 2 ? 2 : k_sel);
    Cand* b = buf[w];
    for (int e = lane; e < n; e += 64) {
        Cand c{-INFINITY, kEmptyId};
        if (e < k_sel) {
            const int64_t id = sel_ids[q * k_sel + e];
            if (id >= 0) {
                const int64_t pos = id - id_offset;
                const float* xr = x_aug + pos * ld_x;
                const float xn = seq_dot(xr, xr, d);
                const float ip = seq_dot(qr, xr, d);
                float dis = (qn + xn) - 2.f * ip;
                dis = dis < 0.f ? 0.f : dis;
                c = Cand{-dis, static_cast<uint32_t>(pos)};
            }
        }
        b[e] = c;
    }
    wave_lds_sync();
    wave_sort_lds(b, n);
    for (int e = lane; e < k; e += 64) {
        const Cand c = b[e];
        const bool ok = c.i != kEmptyId;
        scores[q * k + e] = ok ? -c.s : FLT_MAX;
        ids[q * k + e] = ok ? static_cast<int64_t>(c.i) + id_offset : -1;
    }
    if (unverified && lane == 0) {
        // certificate: an unselected item y has selection score ŝ_y <= s_last, so
        // its distance ‖q‖² − 2·s_y is at least qn − 2·s_last minus the rounding of
        // the selection score and of the reported distance. An item that can
        // compete with the k-th distance has ‖x‖ ≈ ‖q‖, so every term is bounded
        // by scale = 2·qn + 2|s_last| + d_k; the bound allows (d + 4) roundings
        // of that scale, 8x over. A short selection (the whole eligible corpus
        // was selected) needs no certificate.
        int flag = 0;
        if (sel_scores && k_sel > k && sel_ids[q * k_sel + k_sel - 1] >= 0) {
            const float s_last = sel_scores[q * k_sel + k_sel - 1];
            const Cand ck = b[k - 1];
            const float d_k = ck.i != kEmptyId ? -ck.s : FLT_MAX;
            const float gap = (qn - 2.f * s_last) - d_k;
            const float scale = 2.f * qn + 2.f * fabsf(s_last) + d_k;
            const float tol = 8.f * static_cast<float>(d + 4) * 1.1920929e-07f * scale;
            flag = !(gap > tol);
        } else if (k_sel == k && sel_ids[q * k_sel + k_sel - 1] >= 0) {
            flag = 1;  // no over-selection and a full list: nothing certifies the k-th
        }
        unverified[q] = flag;
    }
}

}  // namespace l2
}  // namespace rt

using namespace rt;

extern "C" int rt_l2_augment_f32(const float* x, int64_t n, int d, float* out, int ld_out, int role, void* stream) {
    if (n < 0 || d <= 0 || ld_out < d + 1 || (role != 0 && role != 1)) return RT_ERR_INVALID;
    if (n == 0) return RT_OK;
    if (!x || !out) return RT_ERR_INVALID;
    hipLaunchKernelGGL(l2::augment_kernel, dim3(static_cast<unsigned>((n + 3) / 4)), dim3(256), 0,
                       as_stream(stream), x, n, d, out, ld_out, role);
    return check_launch("l2_augment_kernel");
}

extern "C" int rt_l2_finish_f32(const float* q_aug, int ld_q, const float* x_aug, int ld_x, int d, int64_t nq,
                                int k_sel, const int64_t* sel_ids, const float* sel_scores, int k, float* scores,
                                int64_t* ids, int32_t* unverified, int64_t id_offset, void* stream) {
    if (nq < 0 || d <= 0 || k <= 0 || k_sel < k || ld_q < d || ld_x < d || id_offset < 0) return RT_ERR_INVALID;
    if (k_sel > l2::kFinishN) return RT_ERR_UNSUPPORTED;
    if (nq == 0) return RT_OK;
    if (!q_aug || !x_aug || !sel_ids || !scores || !ids) return RT_ERR_INVALID;
    if (sel_ids == ids && k_sel != k) return RT_ERR_INVALID;  // in place only without over-selection
    hipLaunchKernelGGL(l2::finish_kernel, dim3(static_cast<unsigned>((nq + 3) / 4)), dim3(256), 0, as_stream(stream),
                       q_aug, ld_q, x_aug, ld_x, d, nq, k_sel, sel_ids, sel_scores, k, scores, ids, unverified,
                       id_offset);
    return check_launch("l2_finish_kernel");
}
