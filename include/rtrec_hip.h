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
 * queries [nq, d], items [nx, d], both `dtype`, rows 16-byte aligned:
 * f32: d % 4 == 0, d <= 256; f16/bf16: d % 8 == 0, d <= 256; 1 <= k <= 512;
 * nx + id_offset < 2^32 - 1.
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

/* Corpus-sharded search with ONE corpus-wide threshold per query (several
 * GPUs, each holding a row shard of the corpus that faiss.IndexFlatIP.search
 * would scan whole, src/serving/retrieval.py:141-197): every rank samples its
 * shard, the ranks' samples give each query a threshold that is, w.h.p., at
 * most its k-th score over the WHOLE corpus, and each rank keeps only its
 * rows at or above it — so a query's candidates per shard shrink with the
 * number of shards instead of staying ~k per shard.
 *   rt_flatip_topk_shard_sample: top32 [nq][32] = per query the union of each
 *     lane half's 16 largest group maxima (max of 16 rows) over every
 *     stride-th 128-row stage of the shard, merged and sorted descending
 *     (-inf padded): a subset of the 32 largest sampled group maxima, so a
 *     threshold taken from it is <= the one the exact 32 would give (safe:
 *     only more candidates). stage_counts = {sampled stages, stages} of this
 *     shard.
 *   rt_flatip_topk_shard_plan: host only (no device work): RT_OK and the
 *     stage_counts rt_flatip_topk_shard_sample would report for a shard of
 *     nx rows, or RT_ERR_UNSUPPORTED when the shape has no v4 plan — so every
 *     rank can derive every shard's counts (and whether the global-threshold
 *     path applies on all of them) from the shard sizes alone, without a
 *     collective or a device->host read.
 *   rt_topk_sample_rank: the failure-safe rank (P(threshold > k-th) < 1e-6)
 *     for the sampled fraction sum(sampled) / sum(stages) over all shards
 *     (0 = none fits: search from -inf).
 *   rt_topk_sample_threshold: thr[q] = the rank-th largest of the union of
 *     n_lists (<= 64) such lists (layout [n_lists][nq][32], e.g. all-gathered
 *     over ranks); -FLT_MAX when the union has fewer finite entries.
 *   rt_flatip_topk_shard_search: this shard's rows with score >= thr[q], the
 *     best k of them per query in (score desc, id asc) order, padded with
 *     (-FLT_MAX, -1) when fewer pass. The caller merges the shards' lists;
 *     a query whose merged list holds < min(k, corpus rows) entries had a
 *     threshold above its k-th and is searched again from -inf.
 * f16/bf16 with d % 8 == 0, d <= 128, k <= 128, one query chunk (the v4
 * kernel plan of rt_flatip_topk); RT_ERR_UNSUPPORTED otherwise. The
 * workspace (rt_flatip_topk_shard_workspace_bytes, 0 = unsupported) serves
 * both the sample and the search of the same shape. */
size_t rt_flatip_topk_shard_workspace_bytes(int64_t nq, int64_t nx, int d, int dtype, int k);
int rt_flatip_topk_shard_plan(int64_t nq, int64_t nx, int d, int dtype, int k, int stride, int64_t* stage_counts);
int rt_flatip_topk_shard_sample(const void* queries, int64_t nq, const void* items, int64_t nx, int d, int dtype,
                                int k, int stride, float* top32, int64_t* stage_counts, void* workspace,
                                size_t workspace_bytes, void* stream);
int rt_topk_sample_rank(int k, int64_t sampled_stages, int64_t stages, int* rank);
int rt_topk_sample_threshold(const float* lists, int n_lists, int64_t nq, int rank, float* thr, void* stream);
int rt_flatip_topk_shard_search(const void* queries, int64_t nq, const void* items, int64_t nx, int d, int dtype,
                                int k, const float* thr, int64_t id_offset, float* out_scores, int64_t* out_ids,
                                void* workspace, size_t workspace_bytes, void* stream);

/* Planner override of rt_flatip_topk (tests and tuning; process-wide, not
 * thread-safe, results unchanged by any setting). v4_mode: 0 automatic, 1 never
 * the sampled-threshold kernel pair, 2 it wherever legal (16-bit, d <= 128,
 * k <= 128); + 4: per-split thresholds instead of one corpus-wide threshold
 * per query when the items are split; + 8: fp32 corpora of <= 4096 rows keep
 * the fused register-list scan instead of the score-slab GEMM + per-query
 * select pair (the default for them); + 16: a corpus-wide threshold is
 * sampled by every block over the whole corpus (the round-4 form) instead of
 * by one sample-only launch over every split and a per-query threshold pass.
 * v4_stride: sample every stride-th 128-row stage (0 = planner).
 * v4_rank: threshold = rank-th largest sampled group maximum (-1 = planner,
 * 0 = no sample: a running threshold from -inf). Set before sizing the
 * workspace. */
int rt_flatip_topk_tuning(int v4_mode, int v4_stride, int v4_rank);

/* IndexFlatL2 mode (FaissIndex with metric != "cosine", src/serving/retrieval.py:
 * 96-100). rt_l2_augment_f32 writes rows [x, a, 0...] of ld_out >= d + 1 floats:
 * a = 1 for queries (role 0), a = -0.5*||x||^2 for items (role 1; ||x||^2 a
 * sequential fmaf chain); then rt_flatip_topk on the augmented rows (d' =
 * ld_out) ranks items by q.x - ||x||^2/2, i.e. by ascending ||q - x||^2.
 * rt_l2_finish_f32 takes k_sel >= k such candidates per query (sel_ids
 * [nq, k_sel], item index + id_offset into x_aug, -1 = none) and writes the k
 * nearest by Faiss's reported distance (||q||^2 + ||x||^2 - 2 q.x over the first
 * d columns, sequential fmaf norms and dot, clamped at 0), sorted by (distance
 * asc, id asc), into scores/ids [nq, k]; unfilled slots (FLT_MAX, -1). The
 * selection score and the reported distance round differently: exact (equal to
 * Faiss) unless more than k_sel - k items lie within rounding of the k-th
 * distance. With sel_scores ([nq, k_sel], the selection scores rt_flatip_topk
 * returned with sel_ids) and unverified (int32 [nq]) both given, the finish
 * certifies each query: unverified[q] = 0 when no unselected item can reach
 * the k-th distance within a rounding bound, 1 otherwise (the caller then
 * re-selects that query with a larger k_sel). k_sel <= 512; sel_ids may alias
 * ids only when k_sel == k. */
int rt_l2_augment_f32(const float* x, int64_t n, int d, float* out, int ld_out, int role, void* stream);
int rt_l2_finish_f32(const float* q_aug, int ld_q, const float* x_aug, int ld_x, int d, int64_t nq, int k_sel,
                     const int64_t* sel_ids, const float* sel_scores, int k, float* scores, int64_t* ids,
                     int32_t* unverified, int64_t id_offset, void* stream);

/* Merge n_lists candidate lists per query, layout [n_lists][nq][k_in] (as an
 * all_gather_into_tensor over ranks produces), into the (score desc, id asc)
 * top k_out. id -1 entries are ignored; ids must be < 2^32 - 1; k_out <= 512. */
int rt_topk_merge(const float* scores, const int64_t* ids, int64_t nq, int n_lists, int k_in,
                  int k_out, float* out_scores, int64_t* out_ids, void* stream);

/* On-device negative sampling (sample_negative_items, src/data/movielens.py:
 * 488-512, called per sample by src/training/datasets/movielens.py:104-108).
 * Per row r: num_neg distinct items uniform over [0, num_items) minus the
 * positives of user users[r] (CSR: pos_items[pos_offsets[u] .. pos_offsets[u+1])
 * sorted ascending, unique); if that pool has <= num_neg items, the pool in
 * increasing order followed by -1. Counter-based RNG: the draw is a pure
 * function of (seed + *seed_offset, row, slot, round). num_neg <= 64,
 * num_items < 2^31. out [n, num_neg] int64. */
int rt_sample_negatives(const int64_t* pos_offsets, const int32_t* pos_items, int64_t n_users,
                        const int64_t* users, int64_t n, int64_t num_items, int num_neg, uint64_t seed,
                        const uint64_t* seed_offset, int64_t* out, void* stream);

/* Device batch cursor of a graph-captured epoch (rtrec_amd FeederGraph; the
 * DataLoader batches of src/training/datasets/movielens.py:86-134 over a
 * shuffled interaction list). state = int64 [2] device {batch cursor b,
 * sampler salt}. rt_feeder_batch: row t < batch of batch b is interaction
 * order[b·batch + t]: users[t] = inter_u[row], pos[t] = inter_m[row]
 * (order holds >= (b+1)·batch entries). rt_feeder_commit (one thread, after
 * the step): losses[b] = loss[0], then b += 1 and salt += 1 (the salt is the
 * seed_offset of the batch's rt_sample_negatives). */
int rt_feeder_batch(const int64_t* order, const int64_t* inter_u, const int64_t* inter_m, const int64_t* state,
                    int64_t batch, int64_t* users, int64_t* pos, void* stream);
int rt_feeder_commit(const double* loss, double* losses, int64_t n_losses, int64_t* state, void* stream);

/* ------------------------------------------------------------------------
 * Tower MLP (src/models/two_tower.py:56-72,98-134,196-212,238-281):
 * hidden block l = Linear → act → BatchNorm1d → Dropout, final Linear, then
 * F.normalize(p=2, eps=1e-12).
 *
 * rt_linear_fwd_f32 computes one Linear with fused prologue/epilogue:
 *   A row r  = src[ids ? ids[r] : r]                  (ids: fused row gather)
 *   prev_mode 0: a = A (raw input)
 *             1: a = drop(bn(act_prev(A))), BN in train mode: batch mean/biased var
 *                from prev_stats (fp64 [2k]: Σ act_prev(z), Σ act_prev(z)^2 over m
 *                rows), eps; block 0 writes save_mean/save_invstd [k] and updates
 *                running_mean/var (momentum, unbiased var) — BatchNorm1d.train()
 *             2: same with running stats (eval); block 0 writes save_mean/invstd
 *             3: a = drop(act_prev(A))   (no BN: ItemTower.content_projection)
 *   drop: keep with prob 1-p, scale 1/(1-p), mask = hash(drop_seed, r, col)
 *   z = a · Wᵀ + bias   (W [n, k] row-major, n <= 512)  → z_out [m, n]
 *   stats_out (caller-zeroed) += (Σ_r act(z), Σ_r act(z)^2)
 *   l2_out: F.normalize(z, p=2, eps=1e-12) rows, norms_out[r] = ||z[r]||
 *
 * BatchNorm column sums (stats_out / prev_stats / g_stats / g_prev_stats) are
 * fp64 [RT_STAT_SLOTS][2][width]: row block b adds its partial sums into slot
 * b % RT_STAT_SLOTS (bounds same-address atomic contention), consumers sum the
 * slots in slot order. Caller zeroes them before the producing launch.
 * ------------------------------------------------------------------------ */
#ifndef RT_STAT_SLOTS
#define RT_STAT_SLOTS 8
#endif
#if RT_STAT_SLOTS > 15
#error "RT_STAT_SLOTS > 15: the host arenas (rtrec_amd/models/fused.py STAT_SLOTS) hold 16 slot rows, one of them for ticket counters"
#endif

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
    int prev_mode;           /* 0 raw, 1 BN train, 2 BN eval, 3 act+dropout only        */
    int prev_act;            /* rt_act of the previous block                           */
    const double* prev_stats;/* [RT_STAT_SLOTS][2k] fp64 sums (mode 1)                 */
    const float* bn_gamma;   /* [k]                                                    */
    const float* bn_beta;    /* [k]                                                    */
    float* running_mean;     /* [k] read (mode 2) / updated (mode 1, may be NULL)      */
    float* running_var;      /* [k]                                                    */
    float* save_mean;        /* [k] written by block 0 (modes 1,2; may be NULL)        */
    float* save_invstd;      /* [k]                                                    */
    float bn_eps;
    float bn_momentum;
    float drop_p;            /* dropout prob of the previous block (0 = off)           */
    uint64_t drop_seed;      /* mask seed = drop_seed + (*seed_offset if non-NULL)      */
    const uint64_t* seed_offset; /* device counter (hipGraph replay draws new masks)   */
    float* z_out;            /* [m, n] pre-activation, or NULL                         */
    int act;                 /* activation of THIS block (for stats_out)               */
    double* stats_out;       /* [RT_STAT_SLOTS][2n] accumulated (NULL = skip)          */
    float* l2_out;           /* [m, n] normalized rows (final layer) or NULL          */
    float* norms_out;        /* [m] row norms (with l2_out)                            */
    int64_t* num_batches_tracked; /* prev BN counter, +1 by block 0 in mode 1 (may be NULL) */
    int64_t seg_split;       /* 0, or a multiple of 32 in (0, m): rows [0, seg_split) and
                                [seg_split, m) are two SEPARATE BatchNorm batches (two tower
                                calls — e.g. positives then negatives through the item
                                tower — in one launch). Every per-column BN buffer above and
                                below (prev_stats, save_mean/invstd, stats_out) is then
                                [2][...] (segment-major), running stats are updated segment 0
                                then segment 1, num_batches_tracked += 2. */
    double* zero_buf;        /* optional fp64 [zero_words] set to 0 by the launch before any
                                other work (a step's first launch clears the next
                                accumulators: loss triple, per-tensor grad norms) */
    int64_t zero_words;
    float* wt_out;           /* optional [k, n]: the launch also writes Wᵀ (row kk = column kk
                                of w), which the backward's dz launch reads as rt_linear_bwd_args.wt
                                (NULL = skip) */
    float* a_out;            /* optional [m, k] (k % 4 == 0, 16-B aligned): the launch also writes
                                the transformed input rows it stages (after the previous block's
                                act / BN / dropout prologue and the gather), which the backward's
                                dW launch reads as rt_linear_bwd_args.a_in (NULL = skip) */
    /* BatchNorm finalised by its producer (optional; with stats_out, a training BN after this
     * Linear): the launch's last block per argument set — found by a ticket counter at word
     * nseg·RT_STAT_SLOTS·2n of stats_out (past the slots; caller-zeroed with them) — turns the
     * column sums into the batch mean / invstd and the running-stat updates ONCE, instead of
     * every block of the consuming launch re-deriving them from the fp64 slots. The consuming
     * launch then passes prev_final = 1 and reads them from its save_mean / save_invstd. */
    float* fin_save_mean;    /* [nseg][n] batch means (the consumer's save_mean); NULL = no finalisation */
    float* fin_save_invstd;  /* [nseg][n] 1/sqrt(biased var + eps) */
    float* fin_running_mean; /* [n] momentum update, segment 0 then segment 1 (NULL = skip) */
    float* fin_running_var;  /* [n] with the unbiased batch variance */
    int64_t* fin_num_batches_tracked; /* += nseg (NULL = skip) */
    float fin_eps;
    float fin_momentum;
    int prev_final;          /* prev_mode 1 only: 1 = the producing launch finalised the batch
                                statistics (save_mean / save_invstd hold them; prev_stats, the
                                running stats and num_batches_tracked are not touched here) */
    /* Split-weight planes (DESIGN.md §5 note i): the three bf16 pieces (hi, mid, lo; split3) of a
     * weight, computed ONCE per step by a side task of an earlier launch instead of in registers
     * by every block that uses it. The pieces are the same bits split3 gives, so results are
     * bit-identical to the in-register split. */
    const uint16_t* w_planes;     /* optional [3][n][k] pieces of THIS launch's w (k % 8 == 0, n <= 128,
                                     16-B aligned): the MFMA k-loop reads them (NULL = split w) */
    uint16_t* wt_planes_out;      /* optional [3][k][n]: side task, the pieces of Wᵀ, read by the
                                     backward's dz launch as rt_linear_bwd_args.wt_planes */
    const float* next_w;          /* optional side task: the pieces of another weight [next_n][next_k]
                                     (the next layer's w, for its launch's w_planes; next_k % 8 == 0) */
    uint16_t* next_w_planes;      /* [3][next_n][next_k] */
    int next_n;
    int next_k;
} rt_linear_fwd_args;

int rt_linear_fwd_f32(const rt_linear_fwd_args* args, void* stream);

/* Backward of one Linear and of the block that produced its output gradient.
 *   grad_mode 0: dz = normalize_bwd(dout; l2_out, norms)            (final layer)
 *             1: dz = act'(z)·γ·invstd·(g − Σg/m − x̂·Σg·x̂/m)    (BN train; g_stats)
 *             2: dz = act'(z)·γ·invstd·g                         (BN eval)
 *             3: dz = act'(z)·g                                   (no BN)
 *      with g = d loss/d(BN output) [m, n], x̂ = (act(z) − save_mean)·save_invstd.
 *   dz_ws [m, n] receives dz; dbias += Σ_r dz; dw += dzᵀ·a  (fp32 atomics into
 *   caller-zeroed buffers, one per output element per M-split of at most 32),
 *   a = the forward input of this Linear recomputed by the same prologue
 *   (src/ids/prev_* exactly as passed to rt_linear_fwd_f32).
 *   modes 1/2: dgamma += Σ g·x̂, dbeta += Σ g (read from g_stats; atomic, so two
 *   chains of one tower may run concurrently on different streams).
 *   da = dz·W [m, k] then: dsrc = da (if non-NULL; input gradient, layer 1) and/or
 *   g_prev = drop_bwd_prev(da) with g_prev_stats += (Σ g_prev, Σ g_prev·x̂_prev)
 *   (x̂_prev from src with prev_mean/prev_invstd; prev_mode 1/2 only).
 *   n <= 256 and k <= 512. */
typedef struct {
    int64_t m; int k; int n;
    const float* w;          /* [n, k] */
    float* dw;               /* [n, k] accumulated */
    float* dbias;            /* [n] accumulated or NULL */
    float* dz_ws;            /* [m, n] workspace */
    int grad_mode;
    const float* dout;       /* mode 0: [m, n] */
    const float* l2_out;     /* mode 0: [m, n] */
    const float* norms;      /* mode 0: [m] */
    const float* g;          /* modes 1-3: [m, n] */
    const float* z;          /* modes 1-3: [m, n] pre-activation of this block */
    int act;                 /* this block's activation */
    const double* g_stats;   /* modes 1,2: [RT_STAT_SLOTS][2n] (Σg, Σg·x̂) */
    const float* save_mean;  /* [n] */
    const float* save_invstd;/* [n] */
    const float* bn_gamma;   /* [n] */
    float* dgamma;           /* [n] accumulated or NULL */
    float* dbeta;            /* [n] */
    /* the input A of this linear, recomputed exactly as the forward prologue */
    const float* src; int64_t src_rows; int ld_src; const int64_t* ids;
    int prev_mode; int prev_act;
    const float* prev_mean; const float* prev_invstd;   /* prev block save_mean/invstd */
    const float* prev_gamma; const float* prev_beta;
    float prev_drop_p; uint64_t prev_drop_seed; const uint64_t* seed_offset;
    /* outputs towards the previous block */
    float* g_prev;           /* [m, k] or NULL */
    double* g_prev_stats;    /* [RT_STAT_SLOTS][2k] accumulated, caller zeroes (NULL = skip) */
    float* dsrc;             /* [m, k] input grad (first layer), or NULL */
    int64_t seg_split;       /* as in rt_linear_fwd_args: g_stats, save_mean/invstd,
                                prev_mean/invstd and g_prev_stats are then [2][...] */
    double* dbias_slots;     /* optional fp64 [RT_STAT_SLOTS + 1][n], caller-zeroed: the dz launch
                                adds each row block's column sums of dz (slot = block % SLOTS)
                                and the dW launch folds the slots into dbias — bounded
                                same-address contention; NULL = the dW launch sums dz itself.
                                With fuse_dz the dW launch adds its splits' sums into the slots
                                and the last block of each n-tile folds them; row RT_STAT_SLOTS
                                then holds that launch's per-tile ticket counters (uint64) */
    const float* wt;         /* optional [k, n] = Wᵀ of THIS step's w (rt_linear_fwd_args.wt_out):
                                dA = dz·W then reads contiguous rows of it (NULL = columns of w) */
    int fuse_dz;             /* 1: a layer with no dA (g_prev and dsrc NULL), grad_mode 1-3, a
                                piecewise-linear act and n % 4 == 0 (16-B aligned g, z) computes
                                dz inside its dW launch: the dz launch of the pair is then a no-op
                                and dz_ws is NOT written; dbias, dgamma, dbeta come from the dW
                                launch (ignored when the layer does not qualify) */
    const float* a_in;       /* optional [m, k] = rt_linear_fwd_args.a_out of this step: the dW
                                launch reads A from it as is instead of recomputing it from src /
                                ids / prev_* (those still serve the dz launch); NULL = recompute */
    float* dw_part;          /* optional [splits][n][k] fp32 (splits: rt_linear_bwd_dw_splits):
                                the dW launch STORES each row split's tile sum here instead of
                                adding it into dw with atomics; a later launch folds it (fold_*) */
    const float* fold_src;   /* optional side task of this args' dz launch (fold_in 0) or dW launch
                                (fold_in 1): fold_dst[e] += sum over s < fold_splits of
                                fold_src[s * fold_words + e], in s order, e < fold_words — the
                                fold of an EARLIER launch's dw_part (fold_words % 4 == 0) */
    float* fold_dst;
    int64_t fold_words;
    int fold_splits;
    int fold_in;
    const uint16_t* wt_planes; /* optional [3][k][n] split pieces of Wᵀ (rt_linear_fwd_args.wt_planes_out
                                  of THIS step; n % 8 == 0, 16-B aligned): dA = dz·W reads them instead
                                  of splitting wt / w in registers (bit-identical) */
} rt_linear_bwd_args;

int rt_linear_bwd_f32(const rt_linear_bwd_args* args, void* stream);
/* 1 when the dz launch of these (1 or 2) argument sets is a no-op because
 * their dW launch computes dz itself (rt_linear_bwd_args.fuse_dz), else 0 —
 * the caller may then skip the dz call. Host-only, no GPU work. */
int rt_linear_bwd_dz_fused(const rt_linear_bwd_args* args, int n_args);
/* Row splits per argument set that rt_linear_bwd_dw_f32_multi(args, n_args) will
 * use (the planner is joint over the n_args sets): the first dimension of
 * their dw_part buffers. Host-only, no GPU work. */
int rt_linear_bwd_dw_splits(const rt_linear_bwd_args* args, int n_args, int64_t* splits);
/* the two launches of rt_linear_bwd_f32, separately (same arguments, same
 * order on one stream): dz/dgamma/dbeta/dA, then dW/dbias from dz_ws. */
int rt_linear_bwd_dz_f32(const rt_linear_bwd_args* args, void* stream);
int rt_linear_bwd_dw_f32(const rt_linear_bwd_args* args, void* stream);
/* Up to two independent Linears in ONE launch (n_args = 1 or 2; e.g. layer l
 * of the user and of the item tower): the same arguments and results as n_args
 * separate calls, with both layers' work sharing the GPU at once (a replayed
 * hipGraph runs parallel stream branches one after the other, so the two
 * towers' chains only overlap when their launches are merged).
 * Replaces the concurrent UserTower/ItemTower calls of the trainer step
 * (src/training/trainers/two_tower.py:104-137). */
int rt_linear_fwd_f32_multi(const rt_linear_fwd_args* args, int n_args, void* stream);
int rt_linear_bwd_dz_f32_multi(const rt_linear_bwd_args* args, int n_args, void* stream);
int rt_linear_bwd_dw_f32_multi(const rt_linear_bwd_args* args, int n_args, void* stream);

/* ------------------------------------------------------------------------
 * Losses (fp32 scores, fp32 accumulation; bf16/f16 inputs widened on load).
 * rt_twotower_loss_fwd_bwd fuses, for B users u, B positives p, B*n_neg
 * negatives q (row i*n_neg+j belongs to user i):
 *   explicit (contrastive_loss, src/models/two_tower.py:406-451):
 *     pos_i = u_i·p_i/τ + ub + ib ; neg_ij = u_i·q_ij/τ ; CE over [pos_i, neg_i·], label 0
 *   in-batch (in_batch_negative_loss, :453-479): S = U·Pᵀ/τ, CE(S, arange B)
 *   loss = w_explicit·L_explicit + w_in_batch·L_in_batch   (trainer :134)
 * and writes d loss / d{u, p, q} (OVERWRITTEN) and accumulates d loss / d{ub, ib}
 * into d_user_bias / d_item_bias (may be NULL). n_neg = 0: the loss is the
 * in-batch CE alone (weight 1, trainer fallback :136); w_in_batch = 0 skips
 * the in-batch term (contrastive_loss alone).
 * loss_out: fp64 [3] = (loss, L_explicit, L_in_batch), caller zeroes.
 * Workspace: rt_twotower_loss_workspace_bytes(B).
 * ------------------------------------------------------------------------ */
size_t rt_twotower_loss_workspace_bytes(int64_t b, int d);
int rt_twotower_loss_fwd_bwd(const void* u, const void* p, const void* q, int dtype, int64_t b,
                             int d, int n_neg, float inv_tau, const float* user_bias,
                             const float* item_bias, float w_explicit, float w_in_batch,
                             double* loss_out, float* du, float* dp, float* dq, float* d_user_bias,
                             float* d_item_bias, void* workspace, size_t workspace_bytes, void* stream);

/* Forward-only variants (validation, TwoTowerModel.forward(compute_loss=True)). */
int rt_twotower_loss_fwd(const void* u, const void* p, const void* q, int dtype, int64_t b, int d,
                         int n_neg, float inv_tau, const float* user_bias, const float* item_bias,
                         float w_explicit, float w_in_batch, double* loss_out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* compute_similarity (src/models/two_tower.py:380-404): s_i = u_i·v_i·inv_tau (+ub+ib). */
/* In-batch CE of a data-parallel shard (config C5): S = U·Pᵀ/τ over b local
 * users x n_items in-batch items (all ranks' items, gathered), label of user i =
 * item label_offset + i; loss_out += (L, 0, L) with L = mean_i CE_i over the
 * local users (average over ranks for the global mean). du [b, D] and dp
 * [n_items, D] are OVERWRITTEN with d L / d U, d L / d P (du == NULL: forward
 * only). Replaces in_batch_negative_loss (src/models/two_tower.py:453-479) for
 * the sharded case; b == n_items, label_offset == 0 is the reference loss. */
size_t rt_inbatch_loss_workspace_bytes(int64_t b, int64_t n_items, int d);
int rt_inbatch_loss_fwd_bwd(const void* u, const void* p, int dtype, int64_t b, int64_t n_items, int d,
                            int64_t label_offset, float inv_tau, double* loss_out, float* du, float* dp,
                            void* workspace, size_t workspace_bytes, void* stream);

int rt_similarity_f32(const float* u, const float* v, int64_t b, int d, float inv_tau,
                      const float* user_bias, const float* item_bias, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Optimiser (src/training/trainers/two_tower.py:60-64,144) on ONE flat fp32
 * parameter slab (all tower tensors + biases contiguous) and its grad slab:
 * rt_grad_sqnorm: sumsq_out[t] += Σ g² over tensor t = [offsets[t], offsets[t+1])
 *   (offsets: device int64 [n_tensors+1]; sumsq_out fp64, caller zeroes); also
 *   increments the device step / dropout-seed counters when non-NULL (one
 *   thread), so a replayed hipGraph advances them without extra launches.
 * rt_clip_adam_step: clip_grad_norm_(max_norm): coef = min(1, max_norm /
 *   (sqrt(Σ_t sumsq[t]) + 1e-6)); then torch.optim.Adam with L2 weight decay and
 *   bias correction on g·coef. The step count and learning rate are read from
 *   device memory when step_dev / lr_dev are non-NULL (hipGraph replay), else
 *   from `step` / `lr`. The grads are CONSUMED: every element is zeroed after
 *   use, and zero_buf[0, zero_words) (fp64, may be NULL) is zeroed too — the
 *   next step's accumulators start at zero without memset launches.
 * ------------------------------------------------------------------------ */
int rt_grad_sqnorm(const float* grads, const int64_t* offsets, int n_tensors, double* sumsq_out,
                   int32_t* step_counter, int64_t* seed_counter, void* stream);
int rt_clip_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                      int64_t n, const double* sumsq, int n_tensors, float max_norm, float lr,
                      const float* lr_dev, float beta1, float beta2, float eps, float weight_decay,
                      int step, const int32_t* step_dev, double* zero_buf, int64_t zero_words,
                      void* stream);

/* ------------------------------------------------------------------------
 * Offline evaluation (scripts/evaluate_model.py:162-234, src/evaluation/
 * metrics.py:73-228,248-319).
 *
 * rt_exclusion_bitmap: the train-item mask of generate_recommendations
 *   (evaluate_model.py:224-228: `user_scores[train_item] = -inf` for every
 *   train item < num_items) as the exclude_bits operand of rt_flatip_topk.
 *   Row r uses CSR row u = rows ? rows[r] : r (items sorted ascending, unique;
 *   u outside [0, n_csr_rows) = no exclusions); bits [n_rows, words] uint32,
 *   words >= ceil(n_items/32), every word written.
 *
 * rt_rank_metrics: Evaluator.evaluate per query row r. preds [n_rows,
 *   list_len] int64 ranked item ids (-1 pads a ragged list); ground truth =
 *   CSR row gt_rows ? gt_rows[r] : r (sorted unique items; empty = the row is
 *   skipped, valid[r] = 0, like a user without ground truth); optional
 *   exclusions (CSR, same indirection) are removed from the list before
 *   ranking (metrics.py:279-281). k_values: HOST array of n_k ascending
 *   positive ints, n_k <= RT_METRICS_MAX_K. Predictions must not repeat an item.
 *   per_row fp64 [n_rows][4*n_k + 2] = recall@k[n_k], precision@k[n_k],
 *   ndcg@k[n_k], hit_rate@k[n_k], reciprocal rank, average precision
 *   (the reference's per-user functions, accumulated rank-ascending in fp64).
 *   coverage_bits (optional, caller-zeroed, ceil(num_items/32) words): items
 *   of the first max(k) kept predictions of valid rows (metrics.py:287).
 *
 * rt_rank_metrics_reduce: out fp64 [n_cols + 2] = mean of each per_row column
 *   over valid rows (fixed summation order: deterministic), the number of valid
 *   rows, and coverage = popcount(coverage_bits) / num_items (0 when NULL).
 * ------------------------------------------------------------------------ */
#define RT_METRICS_MAX_K 16

int rt_exclusion_bitmap(const int64_t* offsets, const int32_t* items, int64_t n_csr_rows, const int64_t* rows,
                        int64_t n_rows, int64_t n_items, uint32_t* bits, int64_t words, void* stream);
int rt_rank_metrics(const int64_t* preds, int64_t n_rows, int list_len, const int64_t* gt_offsets,
                    const int32_t* gt_items, const int64_t* gt_rows, int64_t n_gt_rows,
                    const int64_t* ex_offsets, const int32_t* ex_items, const int64_t* ex_rows,
                    int64_t n_ex_rows, const int32_t* k_values, int n_k, int64_t num_items,
                    double* per_row, int32_t* valid, uint32_t* coverage_bits, void* stream);
int rt_rank_metrics_reduce(const double* per_row, const int32_t* valid, int64_t n_rows, int n_cols,
                           const uint32_t* coverage_bits, int64_t num_items, double* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RTREC_HIP_H */
