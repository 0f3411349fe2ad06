/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * CPU restatement of Faiss-1.7.4 IndexFlatIP search + normalize_L2 as the
 * reference calls them:
 *   - faiss.normalize_L2      src/serving/retrieval.py:86,167,214
 *   - faiss.IndexFlatIP(d)    src/serving/retrieval.py:96-98
 *   - index.search(q, k)      src/serving/retrieval.py:170-171
 *   - np.dot + train-item mask + argsort[::-1][:k]
 *                             scripts/evaluate_model.py:217-232
 * Faiss is not vendored in the reference (requirements.txt:13 pins
 * faiss-cpu==1.7.4); its published semantics restated here:
 *   - renorm: x *= 1/sqrt(sum x^2) when the sum is > 0 (fvec_renorm_L2);
 *   - exact fp32 inner products, results sorted by score descending;
 *   - a candidate enters the k-heap only if strictly greater than the current
 *     k-th (items scanned in id order), so the LOWER id wins exact ties:
 *     the result is the first k of the list ordered by (score desc, id asc);
 *   - unfilled slots (k > N): label -1, distance -FLT_MAX (CMin::neutral()).
 * Summation order is DEFINED here as a sequential fmaf chain over the
 * dimension (acc = fmaf(a[j], b[j], acc), j ascending, acc starting at 0);
 * the HIP kernels reproduce exactly this order with the f32 MFMA so fp32
 * results are bit-identical. On dyadic inputs every order gives the same bits.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline float half_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal */
            exp = 127 - 15 + 1;
            while ((man & 0x400u) == 0) { man <<= 1; exp--; }
            man &= 0x3ffu;
            bits = sign | (exp << 23) | (man << 13);
        }
    } else if (exp == 31) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp - 15 + 127) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

static inline float bf16_to_float(uint16_t h) {
    uint32_t bits = (uint32_t)h << 16;
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

/* dtype: 0 = f32, 1 = f16, 2 = bf16 (matches include/rtrec_hip.h rt_dtype) */
void orc_to_f32(const void* src, int dtype, int64_t count, float* dst) {
    if (dtype == 0) {
        memcpy(dst, src, (size_t)count * 4);
    } else if (dtype == 1) {
        const uint16_t* s = (const uint16_t*)src;
        for (int64_t i = 0; i < count; ++i) dst[i] = half_to_float(s[i]);
    } else {
        const uint16_t* s = (const uint16_t*)src;
        for (int64_t i = 0; i < count; ++i) dst[i] = bf16_to_float(s[i]);
    }
}

/* faiss.normalize_L2 → fvec_renorm_L2 (retrieval.py:86) */
void orc_renorm_l2(float* x, int64_t n, int d) {
    for (int64_t i = 0; i < n; ++i) {
        float* r = x + i * (int64_t)d;
        float acc = 0.0f;
        for (int j = 0; j < d; ++j) acc = fmaf(r[j], r[j], acc);
        if (acc > 0.0f) {
            const float inv = 1.0f / sqrtf(acc);
            for (int j = 0; j < d; ++j) r[j] *= inv;
        }
    }
}

float orc_dot(const float* a, const float* b, int d) {
    float acc = 0.0f;
    for (int j = 0; j < d; ++j) acc = fmaf(a[j], b[j], acc);
    return acc;
}

/* a better than b under (score desc, id asc); id -1 (sentinel) is worst */
static inline int better(float sa, int64_t ia, float sb, int64_t ib) {
    if (sa != sb) return sa > sb;
    return (uint64_t)ia < (uint64_t)ib;
}

/* min-heap on "better": root = worst kept element */
static void sift_down(float* hs, int64_t* hi, int k, int pos) {
    for (;;) {
        int l = 2 * pos + 1, r = l + 1, w = pos;
        if (l < k && better(hs[w], hi[w], hs[l], hi[l])) w = l;
        if (r < k && better(hs[w], hi[w], hs[r], hi[r])) w = r;
        if (w == pos) return;
        float ts = hs[pos]; hs[pos] = hs[w]; hs[w] = ts;
        int64_t ti = hi[pos]; hi[pos] = hi[w]; hi[w] = ti;
        pos = w;
    }
}

typedef struct { float s; int64_t i; } pair_t;

static int cmp_pair(const void* a, const void* b) {
    const pair_t* x = (const pair_t*)a;
    const pair_t* y = (const pair_t*)b;
    if (better(x->s, x->i, y->s, y->i)) return -1;
    if (better(y->s, y->i, x->s, x->i)) return 1;
    return 0;
}

/*
 * Exact top-k by inner product for queries [q_begin, q_end) of Q (f32 rows,
 * already converted). exclude: optional bitmap, excl_words uint32 per query
 * (bit j of query row q set → item j skipped, scripts/evaluate_model.py:225-228).
 * out_s / out_i: [nq, k] rows for the processed queries.
 */
static void search_range(const float* Q, const float* X, int64_t nx, int d, int k,
                         const uint32_t* excl, int64_t excl_words, int64_t id_offset,
                         float* out_s, int64_t* out_i, int64_t q_begin, int64_t q_end,
                         pair_t* tmp) {
    for (int64_t q = q_begin; q < q_end; ++q) {
        const float* qr = Q + q * (int64_t)d;
        float* hs = out_s + q * (int64_t)k;
        int64_t* hi = out_i + q * (int64_t)k;
        for (int j = 0; j < k; ++j) { hs[j] = -FLT_MAX; hi[j] = -1; }
        const uint32_t* eb = excl ? excl + q * excl_words : NULL;
        for (int64_t x = 0; x < nx; ++x) {
            if (eb && ((eb[x >> 5] >> (x & 31)) & 1u)) continue;
            const float s = orc_dot(qr, X + x * (int64_t)d, d);
            /* strict: enters only if better than the worst kept (heap root) */
            if (better(s, x, hs[0], hi[0])) {
                hs[0] = s; hi[0] = x;
                sift_down(hs, hi, k, 0);
            }
        }
        for (int j = 0; j < k; ++j) { tmp[j].s = hs[j]; tmp[j].i = hi[j]; }
        qsort(tmp, (size_t)k, sizeof(pair_t), cmp_pair);
        for (int j = 0; j < k; ++j) {
            hs[j] = tmp[j].s;
            hi[j] = tmp[j].i < 0 ? -1 : tmp[j].i + id_offset;
        }
    }
}

/*
 * Q: [nq, d], X: [nx, d] in dtype; converted to f32 exactly first.
 * nthreads > 1 uses OpenMP over queries.
 */
int orc_flatip_search(const void* Q, int64_t nq, const void* X, int64_t nx, int d, int dtype,
                      int k, const uint32_t* excl, int64_t excl_words, int64_t id_offset,
                      float* out_s, int64_t* out_i, int nthreads) {
    if (k <= 0 || d <= 0 || nq < 0 || nx < 0) return -1;
    float* qf = (float*)malloc((size_t)(nq > 0 ? nq : 1) * d * 4);
    float* xf = (float*)malloc((size_t)(nx > 0 ? nx : 1) * d * 4);
    if (!qf || !xf) { free(qf); free(xf); return -2; }
    orc_to_f32(Q, dtype, nq * (int64_t)d, qf);
    orc_to_f32(X, dtype, nx * (int64_t)d, xf);
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
    {
        pair_t* tmp = (pair_t*)malloc(sizeof(pair_t) * (size_t)k);
#pragma omp for schedule(dynamic, 16)
        for (int64_t q = 0; q < nq; ++q)
            search_range(qf, xf, nx, d, k, excl, excl_words, id_offset, out_s, out_i, q, q + 1, tmp);
        free(tmp);
    }
    free(qf);
    free(xf);
    return 0;
}

/*
 * IndexFlatL2.search (src/serving/retrieval.py:99-100, metric != "cosine"):
 * Faiss's BLAS-path distance ||q||^2 + ||x||^2 - 2 q.x (exhaustive_L2sqr_blas,
 * clamped at 0), norms and dot as sequential fmaf chains; the k smallest by
 * (distance asc, id asc) — Faiss's max-heap admits only strictly smaller
 * distances, so the lower id wins exact ties; unfilled slots (FLT_MAX, -1).
 * Q [nq, d], X [nx, d] f32.
 */
int orc_flatl2_search(const float* Q, int64_t nq, const float* X, int64_t nx, int d, int k,
                      float* out_s, int64_t* out_i, int nthreads) {
    if (k <= 0 || d <= 0 || nq < 0 || nx < 0) return -1;
    float* xn = (float*)malloc((size_t)(nx > 0 ? nx : 1) * 4);
    if (!xn) return -2;
    for (int64_t x = 0; x < nx; ++x) xn[x] = orc_dot(X + x * (int64_t)d, X + x * (int64_t)d, d);
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
    {
        pair_t* tmp = (pair_t*)malloc(sizeof(pair_t) * (size_t)k);
#pragma omp for schedule(dynamic, 16)
        for (int64_t q = 0; q < nq; ++q) {
            const float* qr = Q + q * (int64_t)d;
            const float qn = orc_dot(qr, qr, d);
            float* hs = out_s + q * (int64_t)k;  /* scores = -distance while selecting */
            int64_t* hi = out_i + q * (int64_t)k;
            for (int j = 0; j < k; ++j) { hs[j] = -FLT_MAX; hi[j] = -1; }
            for (int64_t x = 0; x < nx; ++x) {
                float dis = (qn + xn[x]) - 2.0f * orc_dot(qr, X + x * (int64_t)d, d);
                if (dis < 0.0f) dis = 0.0f;
                if (better(-dis, x, hs[0], hi[0])) {
                    hs[0] = -dis; hi[0] = x;
                    sift_down(hs, hi, k, 0);
                }
            }
            for (int j = 0; j < k; ++j) { tmp[j].s = hs[j]; tmp[j].i = hi[j]; }
            qsort(tmp, (size_t)k, sizeof(pair_t), cmp_pair);
            for (int j = 0; j < k; ++j) {
                const int ok = tmp[j].i >= 0;
                hs[j] = ok ? -tmp[j].s : FLT_MAX;
                hi[j] = ok ? tmp[j].i : -1;
            }
        }
        free(tmp);
    }
    free(xn);
    return 0;
}

/*
 * Merge n_lists candidate lists per query (layout [n_lists][nq][k_in]) into the
 * (score desc, id asc) top k_out. Entries with id -1 are ignored.
 */
int orc_topk_merge(const float* s, const int64_t* ids, int64_t nq, int n_lists, int k_in,
                   int k_out, float* out_s, int64_t* out_i) {
    const int64_t tot = (int64_t)n_lists * k_in;
    pair_t* tmp = (pair_t*)malloc(sizeof(pair_t) * (size_t)(tot > 0 ? tot : 1));
    if (!tmp) return -2;
    for (int64_t q = 0; q < nq; ++q) {
        int64_t c = 0;
        for (int l = 0; l < n_lists; ++l)
            for (int j = 0; j < k_in; ++j) {
                const int64_t off = ((int64_t)l * nq + q) * k_in + j;
                if (ids[off] < 0) continue;
                tmp[c].s = s[off]; tmp[c].i = ids[off]; ++c;
            }
        qsort(tmp, (size_t)c, sizeof(pair_t), cmp_pair);
        for (int j = 0; j < k_out; ++j) {
            if (j < c) { out_s[q * k_out + j] = tmp[j].s; out_i[q * k_out + j] = tmp[j].i; }
            else { out_s[q * k_out + j] = -FLT_MAX; out_i[q * k_out + j] = -1; }
        }
    }
    free(tmp);
    return 0;
}
