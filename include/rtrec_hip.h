/*
 * rtrec_hip.h — C ABI of the MI355X (gfx950) two-tower retrieval hot path.
 *
 * One shared library, librtrec_hip.so, built with hipcc --offload-arch=gfx950.
 * Conventions (all entry points):
 *   - plain device pointers and sizes, no framework types;
 *   - `stream` is a hipStream_t passed as void* (0 = null stream); every call
 *     is stream-ordered, never synchronises, never allocates (caller-owned
 *     workspaces), so calls are capturable in a hipGraph;
 *   - return RT_OK (0) or a negative rt_status; no C++ exception crosses the ABI;
 *   - row-major contiguous matrices unless a leading dimension is given.
 * Each entry names the reference interface it replaces (paths relative to the
 * reference repo yxyxcyx/Real-Time-Recommendation-System-with-Feature-Store).
 */
#ifndef RTREC_HIP_H
#define RTREC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    RT_OK = 0,
    RT_ERR_INVALID = -1,     /* bad argument (null pointer, size, alignment)       */
    RT_ERR_UNSUPPORTED = -2, /* valid but not implemented shape/dtype/k            */
    RT_ERR_WORKSPACE = -3,   /* workspace too small (query *_workspace_bytes)      */
    RT_ERR_HIP = -4          /* a HIP launch/runtime call failed                    */
} rt_status;

typedef enum { RT_F32 = 0, RT_F16 = 1, RT_BF16 = 2 } rt_dtype;

typedef enum {
    RT_ACT_RELU = 0,       /* nn.ReLU            (src/models/two_tower.py:80) */
    RT_ACT_GELU = 1,       /* nn.GELU (erf)      (:81)                         */
    RT_ACT_LEAKY_RELU = 2, /* nn.LeakyReLU(0.1)  (:82)                         */
    RT_ACT_TANH = 3,       /* nn.Tanh            (:83)                         */
    RT_ACT_SIGMOID = 4,    /* nn.Sigmoid         (:84)                         */
    RT_ACT_NONE = 5
} rt_act;

int rt_abi_version(void);
const char* rt_status_string(int status);
/* last HIP error string recorded by a failing call (thread-local) */
const char* rt_last_error(void);

/* ------------------------------------------------------------------------
 * Row gather (HBM-bound).
 * Replaces: numpy fancy indexing `self.user_features[user_idx]`,
 * `self.movie_features[pos_item_idx]`, `self.movie_features[neg_item_indices]`
 * (src/training/datasets/movielens.py:108-116) and the `nn.Embedding` lookup
 * (src/models/two_tower.py:115-119, 257-261).
 * out[r] = table[ids[r] - row_begin] for ids in [row_begin, row_begin+n_rows);
 * other ids produce a zero row and are counted in *oob_count (may be NULL).
 * A sharded table passes its first global row as row_begin.
 * row_bytes: multiple of 4; table/out 4-byte aligned (16 B for the wide path).
 * ------------------------------------------------------------------------ */
int rt_gather_rows(const void* table, int64_t row_begin, int64_t n_rows, int64_t row_bytes,
                   const int64_t* ids, int64_t n_ids, void* out, int32_t* oob_count, void* stream);

/* nn.Embedding backward (padding_idx rows receive no gradient):
 * grad_table[ids[r]] += grad_out[r] for ids != padding_idx (fp32 atomics). */
int rt_scatter_add_rows_f32(float* grad_table, int64_t n_rows, int dim, const int64_t* ids,
                            int64_t n_ids, const float* grad_out, int64_t padding_idx, void* stream);

/* ------------------------------------------------------------------------
 * faiss.normalize_L2 (src/serving/retrieval.py:86,167,214), in place:
 * x[i] *= 1/sqrtf(sum_j x[i][j]^2) when the sum is > 0. The sum is a
 * sequential fmaf chain over j (the order oracle/flatip.c defines).
 * ------------------------------------------------------------------------ */
int rt_l2_renorm_f32(float* x, int64_t n, int d, void* stream);

/* ------------------------------------------------------------------------
 * Brute-force inner-product top-K (faiss.IndexFlatIP.search,
 * src/serving/retrieval.py:96-98,171; and the masked np.dot + argsort of
 * scripts/evaluate_model.py:217-232).
 * queries [nq, d], items [nx, d], both `dtype`; d % 8 == 0, d <= 512; 1 <= k <= 1024.
 * exclude_bits: optional uint32 bitmap [nq, exclude_words]; bit j of row q set
 *   means item j is skipped for query q.
 * Result rows: the first k of the (score desc, id asc) order (lower id wins
 * exact ties, as Faiss's strict heap insertion does); out_ids = item index +
 * id_offset; unfilled slots (k > eligible items) = (-FLT_MAX, -1).
 * fp32 scores are a sequential fmaf chain over d (bit-identical to the oracle).
 * ------------------------------------------------------------------------ */
size_t rt_flatip_topk_workspace_bytes(int64_t nq, int64_t nx, int d, int dtype, int k);
int rt_flatip_topk(const void* queries, int64_t nq, const void* items, int64_t nx, int d, int dtype,
                   int k, const uint32_t* exclude_bits, int64_t exclude_words, int64_t id_offset,
                   float* out_scores, int64_t* out_ids, void* workspace, size_t workspace_bytes,
                   void* stream);

/* Merge n_lists candidate lists per query, layout [n_lists][nq][k_in] (as an
 * all_gather_into_tensor over ranks produces), into the (score desc, id asc)
 * top k_out. id -1 entries are ignored. k_in*n_lists <= 8192, k_out <= 1024. */
int rt_topk_merge(const float* scores, const int64_t* ids, int64_t nq, int n_lists, int k_in,
                  int k_out, float* out_scores, int64_t* out_ids, void* stream);

/* ------------------------------------------------------------------------
 * Tower MLP (src/models/two_tower.py:56-72,98-134,196-212,238-281):
 * hidden block l = Linear → act → BatchNorm1d → Dropout, final Linear, then
 * F.normalize(p=2, eps=1e-12).
 *
 * rt_linear_fwd_f32 computes one Linear with fused prologue/epilogue:
 *   A row r  = src[gather ? ids[r] : r]               (gather: fused row gather)
 *   if prev_mode != 0: a = drop(bn(act_prev(A)))      (previous hidden block)
 *      bn: train (prev_mode=1) batch stats from prev_stats (fp64 [2*k]: sum, sumsq
 *          of act_prev(z) over prev_m rows), biased var, eps; block 0 also writes
 *          save_mean/save_invstd [k] and updates running_mean/var (momentum);
 *          eval (prev_mode=2): running stats.
 *      drop: keep with prob 1-p, scale 1/(1-p), mask = hash(seed, row, col).
 *   z = a · Wᵀ + bias   (W [n, k] row-major)  → z_out [m, n]
 *   if stats_out: stats_out[c] += Σ_r act(z[r,c]), stats_out[n+c] += Σ act(z)^2 (fp64)
 *   if l2_out: l2_out[r] = z[r]/max(||z[r]||, 1e-12), norms_out[r] = ||z[r]||
 * ------------------------------------------------------------------------ */
typedef struct {
    const float* src;        /* [src_rows, ld_src] input rows (features or prev z) */
    int64_t src_rows;        /* rows in src (bounds for gather)                       */
    int ld_src;              /* leading dim of src (>= k)                              */
    const int64_t* ids;      /* optional gather ids [m] (NULL = identity)              */
    int64_t m;               /* output rows                                            */
    int k;                   /* input features                                         */
    int n;                   /* output features                                        */
    const float* w;          /* [n, k]                                                 */
    const float* bias;       /* [n] or NULL                                            */
    /* previous hidden block applied on load */
    int prev_mode;           /* 0 none, 1 BN train, 2 BN eval                          */
    int prev_act;            /* rt_act of the previous block                           */
    const double* prev_stats;/* [2k] fp64 sums (mode 1)                                */
    const float* bn_gamma;   /* [k]                                                    */
    const float* bn_beta;    /* [k]                                                    */
    float* running_mean;     /* [k] updated in mode 1 (may be NULL)                    */
    float* running_var;      /* [k]                                                    */
    float* save_mean;        /* [k] written in mode 1 (for backward)                   */
    float* save_invstd;      /* [k]                                                    */
    float bn_eps;
    float bn_momentum;
    float drop_p;            /* dropout prob of the previous block (0 = off)           */
    uint64_t drop_seed;
    /* outputs */
    float* z_out;            /* [m, n] pre-activation (may be NULL if l2_out)         */
    int act;                 /* activation of THIS block (for stats)                   */
    double* stats_out;       /* [2n] accumulated, caller zeroes (NULL = skip)          */
    float* l2_out;           /* [m, n] normalized rows (final layer) or NULL          */
    float* norms_out;        /* [m] row norms (final layer) or NULL                    */
} rt_linear_fwd_args;

int rt_linear_fwd_f32(const rt_linear_fwd_args* args, void* stream);

/* Backward of one Linear (+ the hidden block that feeds it):
 *   dz source: grad_mode 0 → dz = normalize_bwd(dout, l2_out, norms) (final layer);
 *              grad_mode 1 → dz = act'(z)·BNbwd(g) from g [m,n], z, bn save stats and
 *                            g_stats (fp64 [2n]: Σg, Σg·x̂) (hidden layer, train BN);
 *              grad_mode 2 → same with eval BN (dz = act'(z)·γ·invstd_running·g).
 *   dW += dzᵀ·a, dbias += Σ_r dz   (fp32 atomics into caller-zeroed buffers)
 *   if dgamma: dgamma += Σ g·x̂, dbeta += Σ g (this block's BN params, mode 1/2)
 *   if g_prev: g_prev = drop_bwd(dz·W) [m, k] and g_prev_stats += (Σg, Σg·x̂_prev)
 *              (x̂_prev from prev z with the prev block's saved stats)
 *   if dsrc (first layer only): dsrc = dz·W (input gradient, e.g. embeddings). */
typedef struct {
    /* this layer */
    int64_t m; int k; int n;
    const float* w;          /* [n, k] */
    float* dw;               /* [n, k] accumulated */
    float* dbias;            /* [n] accumulated or NULL */
    int grad_mode;
    const float* dout;       /* mode 0: [m, n] */
    const float* l2_out;     /* mode 0: [m, n] */
    const float* norms;      /* mode 0: [m] */
    const float* g;          /* mode 1/2: [m, n] grad wrt this block's dropout output */
    const float* z;          /* mode 1/2: [m, n] pre-activation of this block */
    int act;                 /* this block's activation */
    const double* g_stats;   /* mode 1: [2n] */
    const float* save_mean;  /* [n] this block's BN batch mean (mode 1) or running mean (2) */
    const float* save_invstd;/* [n] this block's invstd (mode 1) or 1/sqrt(rv+eps) (2) */
    const float* bn_gamma;   /* [n] */
    float* dgamma;           /* [n] accumulated or NULL */
    float* dbeta;            /* [n] */
    float drop_p; uint64_t drop_seed; /* this block's dropout (applied to g already) */
    /* the input A of this linear: recomputed exactly as the forward prologue */
    const float* src; int64_t src_rows; int ld_src; const int64_t* ids;
    int prev_mode; int prev_act;
    const float* prev_mean; const float* prev_invstd;
    const float* prev_gamma; const float* prev_beta;
    float prev_drop_p; uint64_t prev_drop_seed;
    /* outputs towards the previous block */
    float* g_prev;           /* [m, k] or NULL */
    double* g_prev_stats;    /* [2k] accumulated, caller zeroes */
    float* dsrc;             /* [m, k] input grad (first layer), or NULL */
} rt_linear_bwd_args;

int rt_linear_bwd_f32(const rt_linear_bwd_args* args, void* stream);

/* ------------------------------------------------------------------------
 * Losses (fp32 scores, fp32 accumulation; bf16/f16 inputs widened on load).
 * rt_twotower_loss_fwd_bwd fuses, for B users u, B positives p, B*n_neg
 * negatives q (row i*n_neg+j belongs to user i):
 *   explicit (contrastive_loss, src/models/two_tower.py:406-451):
 *     pos_i = u_i·p_i/τ + ub + ib ; neg_ij = u_i·q_ij/τ ; CE over [pos_i, neg_i·], label 0
 *   in-batch (in_batch_negative_loss, :453-479): S = U·Pᵀ/τ, CE(S, arange B)
 *   loss = w_explicit·L_explicit + w_in_batch·L_in_batch   (trainer :134)
 * and writes d loss / d{u, p, q, ub, ib} (grad buffers are OVERWRITTEN, except
 * dbias which is accumulated). n_neg = 0 disables the explicit term.
 * loss_out: fp64 [3] = (loss, L_explicit, L_in_batch), caller zeroes.
 * Workspace: rt_twotower_loss_workspace_bytes(B).
 * ------------------------------------------------------------------------ */
size_t rt_twotower_loss_workspace_bytes(int64_t b, int d);
int rt_twotower_loss_fwd_bwd(const void* u, const void* p, const void* q, int dtype, int64_t b,
                             int d, int n_neg, float inv_tau, const float* user_bias,
                             const float* item_bias, float w_explicit, float w_in_batch,
                             double* loss_out, float* du, float* dp, float* dq, float* dbias,
                             void* workspace, size_t workspace_bytes, void* stream);

/* Forward-only variants (validation, TwoTowerModel.forward(compute_loss=True)). */
int rt_twotower_loss_fwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                         int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                         float w_explicit, float w_in_batch, double* loss_out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* compute_similarity (src/models/two_tower.py:380-404): s_i = u_i·v_i·inv_tau (+ub+ib). */
int rt_similarity_f32(const float* u, const float* v, int64_t b, int d, float inv_tau,
                      const float* user_bias, const float* item_bias, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Optimiser (src/training/trainers/two_tower.py:60-64,144):
 * rt_grad_sqnorm: sumsq_out[t] = Σ g² over tensor t (fp64, caller zeroes) for the
 *   n_tensors slices [offsets[t], offsets[t+1]) of the flat grad buffer.
 * rt_clip_adam_step: coef = min(1, max_norm/(sqrt(Σ_t ||g_t||)+1e-6)) with
 *   ||g_t|| = sqrt(sumsq[t]) (torch clip_grad_norm_ order); then torch.optim.Adam
 *   (L2 weight decay, bias correction) on the flat fp32 param/grad/m/v buffers.
 * ------------------------------------------------------------------------ */
int rt_grad_sqnorm(const float* grads, const int64_t* offsets, int n_tensors, double* sumsq_out,
                   void* stream);
int rt_clip_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                      int64_t n, const double* sumsq, int n_tensors, float max_norm, float lr,
                      float beta1, float beta2, float eps, float weight_decay, int step,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RTREC_HIP_H */
