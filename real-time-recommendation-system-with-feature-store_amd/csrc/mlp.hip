// Tower MLP kernels (fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32).
//
// Replaces the ATen CPU op chain of UserTower/ItemTower.forward
// (src/models/two_tower.py:56-72, 98-134, 196-212, 238-281):
//   addmm → act → batch_norm → dropout  (per hidden block), addmm, F.normalize
// and its autograd backward. Each Linear is ONE forward launch:
//   prologue  : row gather (layer 1) or the previous block's act → BatchNorm
//               (batch stats finalised from fp64 column sums) → dropout,
//               applied while staging A into LDS;
//   MFMA core : 64-row tile × full output width, K streamed in 32-wide chunks;
//   epilogue  : bias, pre-activation store, fp64 column stats of act(z) for the
//               next BatchNorm, or (final layer) the row L2 normalisation.
// Backward is two launches per Linear: (1) dz (normalize/BN/act backward) +
// dgamma/dbeta + dA = dz·W with the previous block's dropout/BN-stat epilogue,
// (2) dW = dzᵀ·A and dbias over M split across blocks, A recomputed by the
// same prologue. BN column sums go to RT_STAT_SLOTS fp64 slots (include/rtrec_hip.h).
#include "rt_common.h"
#include "split3.h"

namespace rt {
namespace mlp {

typedef float f32x16 __attribute__((ext_vector_type(16)));



constexpr float kNormEps = 1e-12f;

// Up to two independent Linears (the user and the item tower's layer l) in ONE
// launch: blocks [0, split) run a0, the rest a1 — the two chains overlap
// without relying on concurrent streams (a replayed hipGraph runs its parallel
// branches one after the other).
struct FwdLaunch {
    rt_linear_fwd_args a0, a1;
    unsigned split;
};
struct BwdLaunch {
    rt_linear_bwd_args a0, a1;
    unsigned split;
    int64_t rps0, rps1;     // dW: rows per split
    unsigned tn0, tk0, tn1, tk1;  // dW: tile grid of each group
    bool vec0, vec1;              // dW: float4 staging loads
    int ngroups;                  // argument sets in this launch (a1 is a copy of a0 when 1)
    unsigned ksplit = 1;          // dz: blocks per row block (dA column parts)
};

// Side task of a dz (which = 0) or dW (which = 1) launch: fold an EARLIER dW
// launch's row-split partial tiles (rt_linear_bwd_args.dw_part → fold_*) into
// its gradient. Work item = (4 words, a group of kFoldG splits); its loads are
// all issued before the adds; one float4 of fp32 atomics per item when the
// splits form several groups (a plain read-add-store when one). Every thread
// of the launch takes items, before the launch's own work.
constexpr int kFoldG = 8;
__device__ __forceinline__ void fold_side(const BwdLaunch& L, int which) {
    const int64_t nt = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const int64_t gt = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (int g = 0; g < L.ngroups; ++g) {
        const rt_linear_bwd_args& f = g ? L.a1 : L.a0;
        if (!f.fold_src || f.fold_in != which || f.fold_splits <= 0) continue;
        const int64_t n4 = f.fold_words / 4;
        const int ng = (f.fold_splits + kFoldG - 1) / kFoldG;
        for (int64_t it = gt; it < n4 * ng; it += nt) {
            const int64_t e = it % n4;
            const int s0 = static_cast<int>(it / n4) * kFoldG;
            float4 v[kFoldG];
#pragma unroll
            for (int j = 0; j < kFoldG; ++j)
                v[j] = s0 + j < f.fold_splits
                           ? reinterpret_cast<const float4*>(f.fold_src + static_cast<int64_t>(s0 + j) * f.fold_words)[e]
                           : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 t = v[0];
#pragma unroll
            for (int j = 1; j < kFoldG; ++j) { t.x += v[j].x; t.y += v[j].y; t.z += v[j].z; t.w += v[j].w; }
            float* d = f.fold_dst + 4 * e;
            if (ng == 1) {
                const float4 o = *reinterpret_cast<const float4*>(d);
                *reinterpret_cast<float4*>(d) = make_float4(o.x + t.x, o.y + t.y, o.z + t.z, o.w + t.w);
            } else {
                atomicAdd(d, t.x); atomicAdd(d + 1, t.y); atomicAdd(d + 2, t.z); atomicAdd(d + 3, t.w);
            }
        }
    }
}


// ---------------------------------------------------------------------------
// phase probe (diagnostic builds only: -DRT_PHASE_PROBE, tools/c2_phase_probe.py)
// Thread 0 of every block stamps the shader clock at phase boundaries and
// the 100 MHz real-time clock at entry and exit; at exit it appends one
// 8-word record [tag<<32 | block, rt_start, m0, m1, m2, end, rt_end, xcc] to a
// device buffer. Product builds compile none of this.
#ifdef RT_PHASE_PROBE
__device__ unsigned long long* g_probe_buf = nullptr;
__device__ unsigned int g_probe_ctr[64];  // sharded by blockIdx % 64 (one counter: same-address atomics serialise)
__device__ unsigned int g_probe_cap = 0;  // records per shard
struct PhaseProbe {
    uint64_t rt0 = 0, t0 = 0, m[4] = {0, 0, 0, 0};
    __device__ __forceinline__ void start() {
        if (threadIdx.x == 0) {
            rt0 = __builtin_amdgcn_s_memrealtime();
            t0 = __builtin_amdgcn_s_memtime();
        }
    }
    __device__ __forceinline__ void mark(int i) {
        if (threadIdx.x == 0) m[i] = __builtin_amdgcn_s_memtime() - t0;
    }
    __device__ __forceinline__ void end(unsigned tag) {
        if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            m[3] = __builtin_amdgcn_s_memtime() - t0;
            const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
            const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
            const unsigned sh = blockIdx.x & 63u;
            const unsigned slot = atomicAdd(&g_probe_ctr[sh], 1u);
            if (slot < g_probe_cap && g_probe_buf) {
                unsigned long long* o = g_probe_buf + (static_cast<uint64_t>(slot) * 64 + sh) * 8;
                o[0] = (static_cast<uint64_t>(tag) << 32) | blockIdx.x;
                o[1] = rt0; o[2] = m[0]; o[3] = m[1]; o[4] = m[2]; o[5] = m[3]; o[6] = rt1; o[7] = xcc;
            }
        }
    }
};
#define RT_PP_DECL PhaseProbe pp_; pp_.start();
#define RT_PP_MARK(i) pp_.mark(i);
#define RT_PP_END(tag) pp_.end(tag);
#else
#define RT_PP_DECL
#define RT_PP_MARK(i)
#define RT_PP_END(tag)
#endif

// Stores of the big per-row activations (z, dz, the next layer's g) are
// write-through (sc1): the lines leave L2 during the kernel instead of in the
// write-back at the kernel boundary (≈ dirty bytes / 6 TB/s per boundary;
// z1 alone is 18.9 MB), at the price of the next kernel reading them from the
// Infinity Cache instead of L2. Same-box A/B of the C2 step, 3 rounds x 200
// steps: 0.2835-0.2840 vs 0.2895-0.2903 ms (profiles/r04_c2_ab_stores.txt).
// -DRT_NO_WT_STORES builds the plain-store form.
#if !defined(RT_NO_WT_STORES)
#define RT_WT_STORES 1
#endif
__device__ __forceinline__ void st_act(float* p, float v) {
#ifdef RT_WT_STORES
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void st_act4(float* p, float4 v) {
#ifdef RT_WT_STORES
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
#else
    *reinterpret_cast<float4*>(p) = v;
#endif
}

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

using fsplit::Pieces;
using fsplit::s16x8;
using fsplit::split8;
using fsplit::mfma3;
using fsplit::split3;

// previous-block transform applied to every A element (forward AND backward
// recompute use this one function, so the recomputed A is bit-identical)
struct Pro {
    int mode;          // 0 raw, 1/2 act+BN(+drop), 3 act(+drop)
    int act;
    float drop_p, drop_scale;
    uint64_t seed;
    const float* scale;  // LDS [k] (modes 1/2)
    const float* shift;
};

__device__ __forceinline__ float pro_apply(const Pro& p, int64_t r, int c, float v) {
    if (p.mode == 0) return v;
    v = act_eval(p.act, v);
    if (p.mode != 3) v = __builtin_fmaf(v, p.scale[c], p.shift[c]);
    if (p.drop_p > 0.f) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
    return v;
}

// (Σ slot[c], Σ slot[w + c]) over the RT_STAT_SLOTS fp64 slots of stride 2w, in
// slot order: all 2·RT_STAT_SLOTS loads are issued before the first add (one
// memory round trip instead of a dependent chain — the slots are written by
// memory-side atomics, so every load is an HBM/MALL latency)
__device__ __forceinline__ void slot_sums(const double* __restrict__ base, int w, int c, double& s1, double& s2) {
    double v1[RT_STAT_SLOTS], v2[RT_STAT_SLOTS];
#pragma unroll
    for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
        v1[sl] = base[static_cast<int64_t>(sl) * 2 * w + c];
        v2[sl] = base[static_cast<int64_t>(sl) * 2 * w + w + c];
    }
    s1 = 0.0;
    s2 = 0.0;
#pragma unroll
    for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
        s1 += v1[sl];
        s2 += v2[sl];
    }
}

__device__ __forceinline__ void bn_affine(float gamma, float beta, float mean, float invstd, float& scale,
                                          float& shift) {
    scale = gamma * invstd;
    shift = __builtin_fmaf(-mean, scale, beta);
}

// Before a last-block ticket: this thread's slot atomics are performed. Every
// value the last block reads was written by device-scope atomics and is read
// back by returning atomics, so no cache writeback is needed — an agent-scope
// release fence here is a buffer_wbl2 (a write-back of the XCD's L2) in every
// block (-DRT_TICKET_WBL2 restores it for A/B builds).
__device__ __forceinline__ void ticket_release() {
#ifdef RT_TICKET_WBL2
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// BatchNorm finalisation by the producing forward launch (rt_linear_fwd_args
// fin_*): every block calls this after its stats atomics; the group's last
// block (ticket counter past the slots) derives the batch mean / invstd of
// each segment from the fp64 slot sums — read by returning atomic adds of 0,
// at the memory side where the slots live — and applies the running-stat
// updates in segment order, with the same arithmetic as the consumer-side
// finalisation below (linear_fwd_kernel, prev_final = 0).
__device__ __forceinline__ void bn_finalize_last(const rt_linear_fwd_args& a, unsigned nblk) {
    __shared__ int last_s;
    const int tid = threadIdx.x, n = a.n;
    const bool two = a.seg_split > 0;
    const int nseg = two ? 2 : 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slot atomics are performed
    __syncthreads();
    if (tid == 0) {
        ticket_release();
        unsigned long long* cnt =
            reinterpret_cast<unsigned long long*>(a.stats_out + static_cast<int64_t>(nseg) * RT_STAT_SLOTS * 2 * n);
        last_s = atomicAdd(cnt, 1ull) == static_cast<unsigned long long>(nblk) - 1ull ? 1 : 0;
    }
    __syncthreads();
    if (!last_s) return;
    for (int c = tid; c < n; c += blockDim.x) {
        for (int sg = 0; sg < nseg; ++sg) {
            const int64_t ms = two ? (sg == 0 ? a.seg_split : a.m - a.seg_split) : a.m;
            double* ps = a.stats_out + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * n;
            double v1[RT_STAT_SLOTS], v2[RT_STAT_SLOTS];
#pragma unroll
            for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
                v1[sl] = atomicAdd(&ps[static_cast<int64_t>(sl) * 2 * n + c], 0.0);
                v2[sl] = atomicAdd(&ps[static_cast<int64_t>(sl) * 2 * n + n + c], 0.0);
            }
            double s1 = 0.0, s2 = 0.0;  // slot order
#pragma unroll
            for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) {
                s1 += v1[sl];
                s2 += v2[sl];
            }
            const double md = s1 / static_cast<double>(ms);
            double vd = s2 / static_cast<double>(ms) - md * md;
            vd = vd > 0.0 ? vd : 0.0;
            const float mean = static_cast<float>(md);
            const float invstd = static_cast<float>(1.0 / sqrt(vd + static_cast<double>(a.fin_eps)));
            const float var_f = static_cast<float>(ms > 1 ? vd * static_cast<double>(ms) / static_cast<double>(ms - 1) : vd);
            a.fin_save_mean[sg * n + c] = mean;
            if (a.fin_save_invstd) a.fin_save_invstd[sg * n + c] = invstd;
            if (a.fin_running_mean) {
                const float mo = a.fin_momentum;
                a.fin_running_mean[c] = (1.f - mo) * a.fin_running_mean[c] + mo * mean;
                a.fin_running_var[c] = (1.f - mo) * a.fin_running_var[c] + mo * var_f;
            }
        }
    }
    if (tid == 0 && a.fin_num_batches_tracked) *a.fin_num_batches_tracked += nseg;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Block = 32 rows x all n columns; the transformed A tile (32 x k) lives in LDS
// as its three bf16 pieces for the whole reduction (A fragments by
// ds_read_b128), W fragments stream straight from L2 (two float4 per lane per
// k-block) and are split in registers; each 16-deep k-block is one bf16 MFMA
// sextet (mfma3); 4 waves split the output columns.
constexpr int FM = 32;  // rows per block

__host__ __device__ __forceinline__ int pad8(int k) { return (k + 31) / 32 * 32; }  // k padded to whole 32-deep iterations

// WPL: the k-loop reads W's split pieces from rt_linear_fwd_args.w_planes
// (TPW == 1, k % 8 == 0) instead of splitting W fragments in registers
template <int TPW, bool KVEC, bool WPL>  // 32-col tiles per wave (n <= 128*TPW); KVEC: k % 4 == 0
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TPW == 1 ? 3 : 2))) void linear_fwd_kernel(FwdLaunch L) {
    static_assert(!WPL || (TPW == 1 && KVEC), "split-weight planes: one-tile waves, k % 4 == 0");
    const bool g1 = blockIdx.x >= L.split;
    const rt_linear_fwd_args& a = g1 ? L.a1 : L.a0;
    const unsigned bid = blockIdx.x - (g1 ? L.split : 0u);
    constexpr int NT = 4 * TPW;  // column tiles in the block
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int k = a.k, n = a.n;
    const int kp = pad8(k), aplane = FM * kp, aw = 3 * aplane / 2;
    // 16-B chunk c of row r sits at chunk c ^ (r & am): the 32 rows of a
    // ds_read_b128 then cover the 64 banks without padding (with a 16-B pad
    // per row the k = 256 tile took 54 KB and 2 blocks per CU instead of 3)
    const int nch = kp / 8, am = ((nch & -nch) < 16 ? (nch & -nch) : 16) - 1;
    float* scale = sm;                   // [kp]
    float* shift = scale + kp;           // [kp]
    float* As = shift + kp;              // A tile as three bf16 planes [3][FM][kp], chunk-swizzled (aw floats)
    uint16_t* const Ap = reinterpret_cast<uint16_t*>(As);
    float* rowpart = As + aw;            // [NT][FM]
    int64_t* srow = reinterpret_cast<int64_t*>(rowpart + NT * FM);  // [FM]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(bid) * FM;
    const int64_t m = a.m;
    // the transformed A values go to LDS as their three bf16 pieces (split3)
    auto put_a = [&](int r, int c, float4 o) {
        // the staged (transformed) row also to a_out for this Linear's dW launch
        if (a.a_out && c < k && row0 + r < m) st_act4(a.a_out + (row0 + r) * k + c, o);
        uint32_t h0, m0, l0, h1, m1, l1;
        split3(o.x, o.y, h0, m0, l0);
        split3(o.z, o.w, h1, m1, l1);
        uint16_t* q = Ap + r * kp + ((((c >> 3) ^ (r & am)) << 3) | (c & 7));
        *reinterpret_cast<uint2*>(q) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(q + aplane) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(q + 2 * aplane) = make_uint2(l0, l1);
    };
    RT_PP_DECL
    if (blockIdx.x == 0 && a.zero_buf)
        for (int64_t e = tid; e < a.zero_words; e += 256) a.zero_buf[e] = 0.0;

    // A-tile fast path (float4 rows, piecewise-linear act): without a row gather
    // the tile's loads are issued HERE, before the BatchNorm finalisation below,
    // so its fp64 slot reads and the tile reads share one memory round trip
    const int vpr = kp / 4;
    const bool vec = (a.ld_src % 4) == 0 && (reinterpret_cast<uintptr_t>(a.src) & 15) == 0;
    const bool fast = vec && (a.k % 4) == 0 && (256 % vpr) == 0 &&
                      (a.prev_mode == 0 || act_is_piecewise_linear(a.prev_act));
    const bool early = fast && !a.ids && 8 * (256 / vpr) >= FM;  // one pass covers the tile
    // Wᵀ for the backward's dz launch (rt_linear_fwd_args.wt_out): the blocks
    // of each group copy its 32x32 tiles of W transposed, tile i on block
    // i mod (the group's blocks) — a group may have fewer row blocks than W
    // has tiles (32 tiles at the C2 layer 2; 8 row blocks for a batch of 256)
    if (a.wt_out) {
        const int tk = (k + 31) / 32, tiles = tk * ((n + 31) / 32);
        const int nblk = static_cast<int>(g1 ? gridDim.x - L.split : L.split);
        for (int wt = static_cast<int>(bid); wt < tiles; wt += nblk) {
            const int n0 = (wt / tk) * 32, k0 = (wt % tk) * 32;
            const int r = tid >> 3, c = (tid & 7) * 4;
            if (n0 + r < n) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (k0 + c + j < k) a.wt_out[static_cast<int64_t>(k0 + c + j) * n + n0 + r] = a.w[static_cast<int64_t>(n0 + r) * k + k0 + c + j];
            }
        }
    }
    // split-weight planes (side tasks, once per step instead of per block):
    // the pieces of Wᵀ for the dz launch, and of the next layer's W for its
    // forward launch — the same bits split3 gives in registers
    if (a.wt_planes_out || a.next_w_planes) {
        const int nblk = static_cast<int>(g1 ? gridDim.x - L.split : L.split);
        if (a.wt_planes_out) {  // element (kk, nn) of Wᵀ = w[nn][kk]; 4 consecutive nn per thread
            const int64_t plane = static_cast<int64_t>(n) * k;
            const int nq = (n + 3) / 4;
            for (int64_t e = static_cast<int64_t>(bid) * 256 + tid; e < static_cast<int64_t>(k) * nq;
                 e += static_cast<int64_t>(nblk) * 256) {
                const int kk = static_cast<int>(e / nq), n0 = static_cast<int>(e % nq) * 4;
                float x[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) x[j] = n0 + j < n ? a.w[static_cast<int64_t>(n0 + j) * k + kk] : 0.f;
                uint32_t h0, m0, l0, h1, m1, l1;
                split3(x[0], x[1], h0, m0, l0);
                split3(x[2], x[3], h1, m1, l1);
                uint16_t* q = a.wt_planes_out + static_cast<int64_t>(kk) * n + n0;
                if (n0 + 4 <= n && (n % 4) == 0) {
                    *reinterpret_cast<uint2*>(q) = make_uint2(h0, h1);
                    *reinterpret_cast<uint2*>(q + plane) = make_uint2(m0, m1);
                    *reinterpret_cast<uint2*>(q + 2 * plane) = make_uint2(l0, l1);
                } else {
                    const uint32_t hv[2] = {h0, h1}, mv[2] = {m0, m1}, lv[2] = {l0, l1};
                    for (int j = 0; j < 4 && n0 + j < n; ++j) {
                        const int sh = 16 * (j & 1);
                        q[j] = static_cast<uint16_t>(hv[j >> 1] >> sh);
                        q[j + plane] = static_cast<uint16_t>(mv[j >> 1] >> sh);
                        q[j + 2 * plane] = static_cast<uint16_t>(lv[j >> 1] >> sh);
                    }
                }
            }
        }
        if (a.next_w_planes) {  // [next_n][next_k] row-major, next_k % 8 == 0: 8 elements per thread
            const int64_t tot8 = static_cast<int64_t>(a.next_n) * a.next_k / 8;
            const float4* src4 = reinterpret_cast<const float4*>(a.next_w);
            s16x8* dst = reinterpret_cast<s16x8*>(a.next_w_planes);
            for (int64_t e = static_cast<int64_t>(bid) * 256 + tid; e < tot8; e += static_cast<int64_t>(nblk) * 256) {
                const float4 u = src4[2 * e], v = src4[2 * e + 1];
                const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                const Pieces pc = split8(x);
                dst[e] = pc.hi;
                dst[e + tot8] = pc.mid;
                dst[e + 2 * tot8] = pc.lo;
            }
        }
    }
    // one-tile waves (every C2 layer but the first) request their first W
    // fragments before the prologue (they do not depend on it), so the L2
    // latency hides behind the A-tile staging (wider waves would spill)
    const float* wrow[TPW];
    bool tile_on[TPW], row_ok[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        tile_on[i] = (w + 4 * i) * 32 < n;  // wave-uniform
        const int nn = (w + 4 * i) * 32 + c32;
        row_ok[i] = nn < n;
        wrow[i] = a.w + static_cast<int64_t>(row_ok[i] ? nn : 0) * k;
    }
    // two 16-deep k-blocks per iteration (kp % 32 == 0; lane half h holds k =
    // kb + 8h .. kb + 8h + 7 of k-block kb); the W fragments of the next
    // iteration are loaded during this one's MFMAs (register double buffer)
    float4 wv[TPW][4], wn[TPW][4];
    auto load_w = [&](int s, float4 (&dst)[TPW][4]) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kk = s + 16 * (j >> 1) + 8 * h + 4 * (j & 1);
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (tile_on[i] && row_ok[i]) {
                    const float* wr = wrow[i] + kk;
                    if constexpr (KVEC) {
                        if (kk < k) v = *reinterpret_cast<const float4*>(wr);
                    } else {
                        if (kk < k) v.x = wr[0];
                        if (kk + 1 < k) v.y = wr[1];
                        if (kk + 2 < k) v.z = wr[2];
                        if (kk + 3 < k) v.w = wr[3];
                    }
                }
                dst[i][j] = v;
            }
    };
    // WPL: the k-block's three pieces straight from the planes (lane half h
    // holds k = kb + 8h .. kb + 8h + 7 of k-block kb, 16 B per piece)
    uint4 pv[2][3], pn[2][3];
    const int64_t wplane = static_cast<int64_t>(n) * k;
    auto load_p = [&](int s, uint4 (&dst)[2][3]) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int kk = s + 16 * b + 8 * h;
            const bool ok = tile_on[0] && row_ok[0] && kk < k;
            const uint16_t* q = a.w_planes + (static_cast<int64_t>(row_ok[0] ? w * 32 + c32 : 0) * k + (ok ? kk : 0));
#pragma unroll
            for (int p = 0; p < 3; ++p)
                dst[b][p] = ok ? *reinterpret_cast<const uint4*>(q + p * wplane) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    if constexpr (WPL) load_p(0, pn);
    else if constexpr (TPW == 1) load_w(0, wn);
    float4 pre[8];
    if (early) {
        const int c = (tid % vpr) * 4, rstep = 256 / vpr, r0 = tid / vpr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + u * rstep;
            const int64_t gr = row0 + r;
            pre[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < FM && c < k && gr < m && gr < a.src_rows)
                pre[u] = *reinterpret_cast<const float4*>(a.src + gr * a.ld_src + c);
        }
    }

    // BatchNorm of the previous block: this block's batch is its row segment;
    // block 0 derives every segment (it owns the save/running-stat writes,
    // applied in segment order like two sequential tower calls) — unless the
    // producing launch finalised the batch statistics already (prev_final):
    // then every block reads its segment's mean / invstd (4 floats a column)
    const bool two = a.seg_split > 0;
    const int my_seg = (two && row0 >= a.seg_split) ? 1 : 0;
    if (a.prev_mode == 1 && a.prev_final) {
        for (int c = tid; c < k; c += 256)
            bn_affine(a.bn_gamma[c], a.bn_beta[c], a.save_mean[my_seg * k + c], a.save_invstd[my_seg * k + c], scale[c],
                      shift[c]);
    } else if (a.prev_mode == 1 || a.prev_mode == 2) {
        const int nseg = two ? 2 : 1;
        for (int c = tid; c < k; c += 256) {
            for (int sg = 0; sg < nseg; ++sg) {
                if (bid != 0 && sg != my_seg) continue;
                const int64_t ms = two ? (sg == 0 ? a.seg_split : m - a.seg_split) : m;
                float mean, invstd, var_f = 0.f;
                if (a.prev_mode == 1) {
                    const double* ps = a.prev_stats + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * k;
                    double s1, s2;  // slot sums in slot order
                    slot_sums(ps, k, c, s1, s2);
                    const double md = s1 / static_cast<double>(ms);
                    double vd = s2 / static_cast<double>(ms) - md * md;
                    vd = vd > 0.0 ? vd : 0.0;
                    mean = static_cast<float>(md);
                    invstd = static_cast<float>(1.0 / sqrt(vd + static_cast<double>(a.bn_eps)));
                    var_f = static_cast<float>(ms > 1 ? vd * static_cast<double>(ms) / static_cast<double>(ms - 1) : vd);
                } else {
                    mean = a.running_mean[c];
                    invstd = static_cast<float>(1.0 / sqrt(static_cast<double>(a.running_var[c]) + a.bn_eps));
                }
                if (sg == my_seg) bn_affine(a.bn_gamma[c], a.bn_beta[c], mean, invstd, scale[c], shift[c]);
                if (bid == 0) {
                    if (c == 0 && a.prev_mode == 1 && a.num_batches_tracked) *a.num_batches_tracked += 1;
                    if (a.save_mean) a.save_mean[sg * k + c] = mean;
                    if (a.save_invstd) a.save_invstd[sg * k + c] = invstd;
                    if (a.prev_mode == 1 && a.running_mean) {
                        const float mo = a.bn_momentum;
                        a.running_mean[c] = (1.f - mo) * a.running_mean[c] + mo * mean;
                        a.running_var[c] = (1.f - mo) * a.running_var[c] + mo * var_f;
                    }
                }
            }
        }
    }
    RT_PP_MARK(0)  // thread 0's BN finalisation done (its early A loads may still be in flight)
    if (tid < FM) {
        const int64_t gr = row0 + tid;
        int64_t sr = -1;
        if (gr < m) {
            sr = a.ids ? a.ids[gr] : gr;
            if (sr < 0 || sr >= a.src_rows) sr = -1;
        }
        srow[tid] = sr;
    }
    __syncthreads();
    const uint64_t seed = a.drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.drop_p, a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f, seed,
                  scale, shift};
    {   // stage the transformed A tile: float4 loads, 4 in flight per thread
        const int total = FM * vpr;
        if (fast) {
            // fast path: 4 fixed columns per thread (BN affine in registers, no
            // per-element division / LDS reads / act switch), rows strided by 256/vpr
            const int c = (tid % vpr) * 4, rstep = 256 / vpr;
            const bool bn = pro.mode == 1 || pro.mode == 2;
            const float4 sc4 = bn ? *reinterpret_cast<const float4*>(scale + c) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float4 sh4 = bn ? *reinterpret_cast<const float4*>(shift + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float sl = act_slope(pro.act);
            const bool drop = pro.drop_p > 0.f;
            for (int r0 = tid / vpr; r0 < FM; r0 += 8 * rstep) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = r0 + u * rstep;
                    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (early) {
                        v[u] = pre[u];
                    } else if (r < FM && c < k) {
                        const int64_t sr = srow[r];
                        if (sr >= 0) v[u] = *reinterpret_cast<const float4*>(a.src + sr * a.ld_src + c);
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = r0 + u * rstep;
                    if (r >= FM) break;
                    const int64_t gr = row0 + r;
                    const bool ok = srow[r] >= 0 && c < k;
                    auto tf = [&](float x, int cc, float scv, float shv) {
                        if (pro.mode == 0) return x;
                        x = act_pwl(sl, x);
                        if (bn) x = __builtin_fmaf(x, scv, shv);
                        if (drop) x = dropout_keep(pro.seed, gr, cc, pro.drop_p) ? x * pro.drop_scale : 0.f;
                        return x;
                    };
                    float4 o;
                    o.x = ok ? tf(v[u].x, c, sc4.x, sh4.x) : 0.f;
                    o.y = ok ? tf(v[u].y, c + 1, sc4.y, sh4.y) : 0.f;
                    o.z = ok ? tf(v[u].z, c + 2, sc4.z, sh4.z) : 0.f;
                    o.w = ok ? tf(v[u].w, c + 3, sc4.w, sh4.w) : 0.f;
                    put_a(r, c, o);
                }
            }
        } else
        for (int base = tid; base < total; base += 256 * 4) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const int64_t sr = srow[r];
                    if (sr >= 0 && c < k) {
                        const float* sp = a.src + sr * a.ld_src + c;
                        if (vec && c + 4 <= k) v[u] = *reinterpret_cast<const float4*>(sp);
                        else {
                            v[u].x = sp[0];
                            if (c + 1 < k) v[u].y = sp[1];
                            if (c + 2 < k) v[u].z = sp[2];
                            if (c + 3 < k) v[u].w = sp[3];
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const bool ok = srow[r] >= 0;
                    const int64_t gr = row0 + r;
                    float4 o;
                    o.x = (ok && c < k) ? pro_apply(pro, gr, c, v[u].x) : 0.f;
                    o.y = (ok && c + 1 < k) ? pro_apply(pro, gr, c + 1, v[u].y) : 0.f;
                    o.z = (ok && c + 2 < k) ? pro_apply(pro, gr, c + 2, v[u].z) : 0.f;
                    o.w = (ok && c + 3 < k) ? pro_apply(pro, gr, c + 3, v[u].w) : 0.f;
                    put_a(r, c, o);
                }
            }
        }
    }
    __syncthreads();
    RT_PP_MARK(1)

    f32x16 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x16{};
    const uint16_t* ap = Ap + c32 * kp;
    const int asw = c32 & am;
    if constexpr (TPW != 1) load_w(0, wn);
    if constexpr (WPL) {
        for (int s = 0; s < kp; s += 32) {
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int p = 0; p < 3; ++p) pv[b][p] = pn[b][p];
            if (s + 32 < kp) load_p(s + 32, pn);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int ao = (((s + 16 * b) >> 3) + h) ^ asw;
                Pieces pa;
                pa.hi = *reinterpret_cast<const s16x8*>(ap + 8 * ao);
                pa.mid = *reinterpret_cast<const s16x8*>(ap + aplane + 8 * ao);
                pa.lo = *reinterpret_cast<const s16x8*>(ap + 2 * aplane + 8 * ao);
                if (tile_on[0]) {
                    const Pieces pb{__builtin_bit_cast(s16x8, pv[b][0]), __builtin_bit_cast(s16x8, pv[b][1]),
                                    __builtin_bit_cast(s16x8, pv[b][2])};
                    acc[0] = mfma3(pa, pb, acc[0]);
                }
            }
        }
    } else
    for (int s = 0; s < kp; s += 32) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) wv[i][j] = wn[i][j];
        if (s + 32 < kp) load_w(s + 32, wn);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int ao = (((s + 16 * b) >> 3) + h) ^ asw;
            Pieces pa;
            pa.hi = *reinterpret_cast<const s16x8*>(ap + 8 * ao);
            pa.mid = *reinterpret_cast<const s16x8*>(ap + aplane + 8 * ao);
            pa.lo = *reinterpret_cast<const s16x8*>(ap + 2 * aplane + 8 * ao);
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                if (!tile_on[i]) continue;
                const float4 u = wv[i][2 * b], v = wv[i][2 * b + 1];
                const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                acc[i] = mfma3(pa, split8(x), acc[i]);
            }
        }
    }

    RT_PP_MARK(2)
    // ---- epilogue ----
    const bool l2 = a.l2_out != nullptr;
    // final layer, fast form: z² staged column-major in the (now idle) A tile,
    // row sums by 8 threads per row (DPP butterfly), one sqrt and one division
    // per row, then a multiply per element — instead of a 32-lane shuffle
    // reduction per row and a division per element
    if (l2 && !a.z_out && !a.stats_out && n * (FM + 1) <= aw) {
        __syncthreads();  // every wave is done reading As
        float* zsq = As;  // [n][FM + 1]
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int col = (w + 4 * i) * 32 + c32;
            if ((w + 4 * i) * 32 >= n) continue;  // wave-uniform
            const bool col_ok = col < n;
            const float b = (col_ok && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
                const float z = acc[i][r] + b;
                acc[i][r] = z;
                if (col_ok) zsq[col * (FM + 1) + lr] = (row0 + lr < m) ? z * z : 0.f;
            }
        }
        __syncthreads();
        {
            const int row = tid >> 3, part = tid & 7;  // 32 rows x 8 threads
            float ss = 0.f;
            for (int c = part; c < n; c += 8) ss += zsq[c * (FM + 1) + row];
            ss += __shfl_xor(ss, 1, 64);
            ss += __shfl_xor(ss, 2, 64);
            ss += __shfl_xor(ss, 4, 64);
            if (part == 0) {
                const float nrm = sqrtf(ss);
                rowpart[row] = 1.f / fmaxf(nrm, kNormEps);
                if (row0 + row < m && a.norms_out) a.norms_out[row0 + row] = nrm;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int col = (w + 4 * i) * 32 + c32;
            if ((w + 4 * i) * 32 >= n) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gr = row0 + lr;
                if (gr < m && col < n) st_act(a.l2_out + gr * n + col, acc[i][r] * rowpart[lr]);
            }
        }
        RT_PP_END(1)
        return;
    }
    double* const stats = a.stats_out ? a.stats_out + (static_cast<int64_t>(my_seg) * RT_STAT_SLOTS +
                                                       bid % RT_STAT_SLOTS) * 2 * n : nullptr;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int ct = w + 4 * i;
        const int col = ct * 32 + c32;
        const bool col_ok = col < n;
        const float b = (col_ok && a.bias) ? a.bias[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
        if (row0 + FM <= m && a.z_out && !l2 && act_is_piecewise_linear(a.act)) {
            // full row block (the C2 hidden layers): no per-element predicates,
            // 32-bit offsets from one base pointer
            if (ct * 32 >= n) continue;  // wave-uniform
            float* zp = a.z_out + (row0 + 4 * h) * n + col;
            const float sl = act_slope(a.act);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float z = acc[i][r] + b;
                if (col_ok) st_act(zp + ((r & 3) + 8 * (r >> 2)) * n, z);
                const float av = act_pwl(sl, z);
                s1 += av;
                s2 += av * av;
            }
            if (!col_ok) s1 = s2 = 0.f;
        } else
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t gr = row0 + lr;
            const float z = acc[i][r] + b;
            acc[i][r] = z;
            const bool ok = col_ok && gr < m;
            if (ok && a.z_out) st_act(a.z_out + gr * n + col, z);
            if (ok && stats) {
                const float av = act_eval(a.act, z);
                s1 += av;
                s2 += av * av;
            }
            if (l2) {
                float q = ok ? z * z : 0.f;
#pragma unroll
                for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
                if (c32 == 0) rowpart[ct * FM + lr] = q;
            }
        }
        if (stats) {
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (h == 0 && col_ok) {
                atomicAdd(&stats[col], static_cast<double>(s1));
                atomicAdd(&stats[n + col], static_cast<double>(s2));
            }
        }
    }
    if (stats && a.fin_save_mean) bn_finalize_last(a, g1 ? gridDim.x - L.split : L.split);
    if (l2) {
        __syncthreads();
        const int nt_used = (n + 31) / 32;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int col = (w + 4 * i) * 32 + c32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gr = row0 + lr;
                if (gr < m && col < n) {
                    float ss = 0.f;
                    for (int t = 0; t < nt_used; ++t) ss += rowpart[t * FM + lr];  // fixed order
                    const float nrm = sqrtf(ss);
                    a.l2_out[gr * n + col] = acc[i][r] / fmaxf(nrm, kNormEps);
                    if (col == 0 && a.norms_out) a.norms_out[gr] = nrm;
                }
            }
        }
    }
    RT_PP_END(1)
}

// ---------------------------------------------------------------------------
// backward 1: dz, dgamma/dbeta, dA = dz·W (+ g_prev / dsrc epilogue)
// ---------------------------------------------------------------------------
// Block = 32 rows. dz (32 x n) lives in LDS; dA = dz·W reads W[n][k] rows
// coalesced along k straight from L2 (the reduction runs over n).
// (3 waves per SIMD: the C2 launches' 576 blocks need 3 co-resident blocks on
// some CUs; the register cap moves the accumulators from AGPRs to VGPRs, no spill)
// WPL: dA reads Wᵀ's split pieces from rt_linear_bwd_args.wt_planes (n % 8 == 0)
// KS: L.ksplit > 1 (dA columns of a row block split over blocks)
template <int TPWK, bool WPL, bool KS>  // 32-col dA tiles per wave (k <= 128*TPWK)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void linear_bwd_dz_kernel(BwdLaunch L) {
#ifdef RT_FOLD_FIRST
    fold_side(L, 0);
#endif
    // L.ksplit > 1: the dA columns of a row block are split over ksplit blocks
    // (part kpart takes dA tiles kpart·4·TPWK ..), so a launch with fewer row
    // blocks than CUs still fills the chip; phase A's side effects (dz_ws, the
    // dbias slots, dgamma/dbeta) belong to part 0
    const unsigned kpart = KS ? blockIdx.x % L.ksplit : 0u, bx = KS ? blockIdx.x / L.ksplit : blockIdx.x;
    const bool prim = kpart == 0;
    const int tb = static_cast<int>(kpart) * 4 * TPWK;  // first dA column tile of this block
    const bool g1 = bx >= L.split;
    const rt_linear_bwd_args& a = g1 ? L.a1 : L.a0;
    const unsigned bid = bx - (g1 ? L.split : 0u);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int np = pad8(n), ldz = np + 4;
    float* Dz = sm;  // [FM][ldz]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(bid) * FM;
    const bool two = a.seg_split > 0;
    const int my_seg = (two && row0 >= a.seg_split) ? 1 : 0;
    const int64_t seg_m = two ? (my_seg == 0 ? a.seg_split : m - a.seg_split) : m;
    RT_PP_DECL

    // one-tile waves request dA's first W fragments here, ahead of phase A
    // (they do not depend on it), so their latency hides behind the dz tile.
    // One 16-deep k-block (bf16 MFMA sextet) per iteration: lane half h holds
    // n = kb + 8h .. kb + 8h + 7; the next k-block's W loaded during this one's MFMAs
    float wv[TPWK][8], wn[TPWK][8];
    // (the W pointer read once: inside the conditional loads below a field of
    // the selected launch group was re-loaded from the kernarg segment per load)
    const float* __restrict__ Wt = a.w;
    // with Wᵀ (a.wt, n % 8 == 0) a lane's 8 consecutive n of column kk are one
    // contiguous 32-byte run: two float4 loads instead of eight strided ones
#ifdef RT_NO_WT_ROWS  // A/B variant: the strided column loads of w
    const float* __restrict__ WtT = nullptr;
#else
    const float* __restrict__ WtT = (a.wt && (n % 8) == 0) ? a.wt : nullptr;
#endif
    auto load_w = [&](int s, float (&dst)[TPWK][8]) {
#pragma unroll
        for (int i = 0; i < TPWK; ++i) {
            const int kk = (tb + w + 4 * i) * 32 + c32;
            const bool on = (tb + w + 4 * i) * 32 < k && kk < k;
            if (WtT) {
                const int nn = s + 8 * h;
                float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
                if (on && nn < n) {
                    const float* p = WtT + static_cast<int64_t>(kk) * n + nn;
                    v0 = *reinterpret_cast<const float4*>(p);
                    v1 = *reinterpret_cast<const float4*>(p + 4);
                }
                dst[i][0] = v0.x; dst[i][1] = v0.y; dst[i][2] = v0.z; dst[i][3] = v0.w;
                dst[i][4] = v1.x; dst[i][5] = v1.y; dst[i][6] = v1.z; dst[i][7] = v1.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int nn = s + 8 * h + j;
                    dst[i][j] = (on && nn < n) ? Wt[static_cast<int64_t>(nn) * k + kk] : 0.f;
                }
            }
        }
    };
    // WPL: per tile and k-block the three pieces of Wᵀ[kk][nn .. nn + 7], 16 B each
    uint4 pv[TPWK][3], pn[TPWK][3];
    const uint16_t* __restrict__ WtP = a.wt_planes;
    const int64_t tplane = static_cast<int64_t>(k) * n;
    auto load_p = [&](int s, uint4 (&dst)[TPWK][3]) {
#pragma unroll
        for (int i = 0; i < TPWK; ++i) {
            const int kk = (tb + w + 4 * i) * 32 + c32;
            const int nn = s + 8 * h;
            const bool ok = (tb + w + 4 * i) * 32 < k && kk < k && nn < n;
            const uint16_t* q = WtP + (ok ? static_cast<int64_t>(kk) * n + nn : 0);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                dst[i][p] = ok ? *reinterpret_cast<const uint4*>(q + p * tplane) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    if constexpr (TPWK == 1) {  // (two-tile waves would spill)
        if (a.g_prev || a.dsrc) {
            if constexpr (WPL) load_p(0, pn);
            else load_w(0, wn);
        }
    }

    // ---- phase A: dz tile ----
    const int l4 = n / 4;  // grad_mode 0 fast path: float4 lanes per row (a power of two <= 64)
    if (a.grad_mode == 0 && (n % 4) == 0 && l4 <= 64 && (l4 & (l4 - 1)) == 0 && np == n) {
        // F.normalize backward, every load of the wave's 8 rows issued up front:
        // l4 lanes per row, 64/l4 rows per pass, segmented lane sums for the dots
        const int rpp = 64 / l4, sub = lane / l4, li = lane % l4, c = 4 * li;
        float4 lv[8], dv[8];
        float nr[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int r = w * 8 + p * rpp + sub;
            const int64_t gr = row0 + r;
            lv[p] = make_float4(0.f, 0.f, 0.f, 0.f);
            dv[p] = lv[p];
            nr[p] = 1.f;
            if (p * rpp < 8 && gr < m) {
                lv[p] = *reinterpret_cast<const float4*>(a.l2_out + gr * n + c);
                dv[p] = *reinterpret_cast<const float4*>(a.dout + gr * n + c);
                nr[p] = a.norms[gr];
            }
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            if (p * rpp >= 8) break;
            const int r = w * 8 + p * rpp + sub;
            const int64_t gr = row0 + r;
            float dot = lv[p].x * dv[p].x + lv[p].y * dv[p].y + lv[p].z * dv[p].z + lv[p].w * dv[p].w;
            for (int o = 1; o < l4; o <<= 1) dot += __shfl_xor(dot, o, 64);
            const bool big = nr[p] > kNormEps;
            const float inv = 1.f / (big ? nr[p] : kNormEps);
            float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gr < m) {
                d.x = big ? (dv[p].x - lv[p].x * dot) * inv : dv[p].x * inv;
                d.y = big ? (dv[p].y - lv[p].y * dot) * inv : dv[p].y * inv;
                d.z = big ? (dv[p].z - lv[p].z * dot) * inv : dv[p].z * inv;
                d.w = big ? (dv[p].w - lv[p].w * dot) * inv : dv[p].w * inv;
                if (prim) st_act4(a.dz_ws + gr * n + c, d);
            }
            *reinterpret_cast<float4*>(Dz + r * ldz + c) = d;
        }
    } else if (a.grad_mode == 0) {
        for (int rr = w * 8; rr < w * 8 + 8; ++rr) {
            const int64_t gr = row0 + rr;
            if (gr < m) {
                float dot = 0.f;
                for (int c = lane; c < n; c += 64) dot += a.l2_out[gr * n + c] * a.dout[gr * n + c];
                dot = wave_sum(dot);
                const float nrm = a.norms[gr];
                const bool big = nrm > kNormEps;
                const float inv = 1.f / (big ? nrm : kNormEps);
                for (int c = lane; c < np; c += 64) {
                    float dz = 0.f;
                    if (c < n) {
                        const float dv = a.dout[gr * n + c];
                        dz = big ? (dv - a.l2_out[gr * n + c] * dot) * inv : dv * inv;
                        if (prim) a.dz_ws[gr * n + c] = dz;
                    }
                    Dz[rr * ldz + c] = dz;
                }
            } else {
                for (int c = lane; c < np; c += 64) Dz[rr * ldz + c] = 0.f;
            }
        }
    } else {
        // per-column BN-backward coefficients, then a float4 elementwise pass
        float* cA = Dz + FM * ldz;   // γ·invstd (mode 1/2) or 1
        float* cB = cA + np;         // Σg/m
        float* cC = cB + np;         // Σg·x̂/m
        float* cM = cC + np;         // mean
        float* cI = cM + np;         // invstd
        const float inv_m = 1.f / static_cast<float>(seg_m);
        const double* gst = a.g_stats ? a.g_stats + static_cast<int64_t>(my_seg) * RT_STAT_SLOTS * 2 * n : nullptr;
        const int vpr = np / 4;
        const bool vec = (n % 4) == 0;
        const bool fast = vec && (256 % vpr) == 0 && act_is_piecewise_linear(a.act) && a.grad_mode != 3;
        // fast path with one pass over the tile: its g loads are issued before
        // the coefficient loads below, so both share one memory round trip (z
        // follows after the barrier: both sets at once would cost occupancy)
        const bool early = fast && 8 * (256 / vpr) >= FM;
        float4 pg[8];
        if (early) {
            const int c = (tid % vpr) * 4, rstep = 256 / vpr, r0 = tid / vpr;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int r = r0 + u * rstep;
                const int64_t gr = row0 + r;
                pg[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (r < FM && gr < m && c < n) pg[u] = *reinterpret_cast<const float4*>(a.g + gr * n + c);
            }
        }
        for (int c = tid; c < np; c += 256) {
            float A = 1.f, Bc = 0.f, C = 0.f, M = 0.f, I = 1.f;
            if (c < n && (a.grad_mode == 1 || a.grad_mode == 2)) {
                I = a.save_invstd[my_seg * n + c];
                M = a.save_mean[my_seg * n + c];
                A = a.bn_gamma[c] * I;
                if (a.grad_mode == 1) {
                    double gs1, gs2;
                    slot_sums(gst, n, c, gs1, gs2);
                    Bc = static_cast<float>(gs1) * inv_m;
                    C = static_cast<float>(gs2) * inv_m;
                }
            }
            cA[c] = A; cB[c] = Bc; cC[c] = C; cM[c] = M; cI[c] = I;
        }
        __syncthreads();
        const int total = FM * vpr;
        if (fast) {
            // fast path: each thread owns 4 fixed columns (coefficients in
            // registers, no per-element division or LDS reads), rows strided by
            // 256/vpr; all g/z loads of the thread issued before the math
            const int c = (tid % vpr) * 4, rstep = 256 / vpr;
            const float4 fA = *reinterpret_cast<const float4*>(cA + c), fB = *reinterpret_cast<const float4*>(cB + c);
            const float4 fC = *reinterpret_cast<const float4*>(cC + c), fM = *reinterpret_cast<const float4*>(cM + c);
            const float4 fI = *reinterpret_cast<const float4*>(cI + c);
            const float sl = act_slope(a.act);
            for (int r0 = tid / vpr; r0 < FM; r0 += 8 * rstep) {
                float4 gv[8], zv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = r0 + u * rstep;
                    const int64_t gr = row0 + r;
                    gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    zv[u] = gv[u];
                    if (early) {
                        gv[u] = pg[u];
                        if (r < FM && gr < m && c < n) zv[u] = *reinterpret_cast<const float4*>(a.z + gr * n + c);
                    } else if (r < FM && gr < m && c < n) {
                        gv[u] = *reinterpret_cast<const float4*>(a.g + gr * n + c);
                        zv[u] = *reinterpret_cast<const float4*>(a.z + gr * n + c);
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = r0 + u * rstep;
                    if (r >= FM) break;
                    const int64_t gr = row0 + r;
                    auto one = [&](float g, float z, float A, float B, float C, float M, float I) {
                        const float xh = (act_pwl(sl, z) - M) * I;
                        return A * (g - B - xh * C) * (z > 0.f ? 1.f : sl);
                    };
                    float4 d;
                    d.x = one(gv[u].x, zv[u].x, fA.x, fB.x, fC.x, fM.x, fI.x);
                    d.y = one(gv[u].y, zv[u].y, fA.y, fB.y, fC.y, fM.y, fI.y);
                    d.z = one(gv[u].z, zv[u].z, fA.z, fB.z, fC.z, fM.z, fI.z);
                    d.w = one(gv[u].w, zv[u].w, fA.w, fB.w, fC.w, fM.w, fI.w);
                    if (gr >= m || c >= n) d = make_float4(0.f, 0.f, 0.f, 0.f);
                    *reinterpret_cast<float4*>(Dz + r * ldz + c) = d;
                    if (prim && gr < m && c < n) st_act4(a.dz_ws + gr * n + c, d);
                }
            }
        } else
        for (int base = tid; base < total; base += 256 * 4) {
            float4 gv[4], zv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                zv[u] = gv[u];
                if (e < total) {
                    const int r = e / vpr, c = (e - r * vpr) * 4;
                    const int64_t gr = row0 + r;
                    if (gr < m && c < n) {
                        const int64_t off = gr * n + c;
                        if (vec) {
                            gv[u] = *reinterpret_cast<const float4*>(a.g + off);
                            zv[u] = *reinterpret_cast<const float4*>(a.z + off);
                        } else {
                            gv[u].x = a.g[off]; zv[u].x = a.z[off];
                            if (c + 1 < n) { gv[u].y = a.g[off + 1]; zv[u].y = a.z[off + 1]; }
                            if (c + 2 < n) { gv[u].z = a.g[off + 2]; zv[u].z = a.z[off + 2]; }
                            if (c + 3 < n) { gv[u].w = a.g[off + 3]; zv[u].w = a.z[off + 3]; }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = base + u * 256;
                if (e >= total) continue;
                const int r = e / vpr, c = (e - r * vpr) * 4;
                const int64_t gr = row0 + r;
                float dzv[4];
                const float gs[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
                const float zs[4] = {zv[u].x, zv[u].y, zv[u].z, zv[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cc = c + j;
                    float dz = 0.f;
                    if (gr < m && cc < n) {
                        const float xh = (act_eval(a.act, zs[j]) - cM[cc]) * cI[cc];
                        const float dr = (a.grad_mode == 3) ? gs[j] : cA[cc] * (gs[j] - cB[cc] - xh * cC[cc]);
                        dz = dr * act_grad_eval(a.act, zs[j]);
                    }
                    dzv[j] = dz;
                }
                *reinterpret_cast<float4*>(Dz + r * ldz + c) = make_float4(dzv[0], dzv[1], dzv[2], dzv[3]);
                if (prim && gr < m && c < n) {
                    const int64_t off = gr * n + c;
                    if (vec) *reinterpret_cast<float4*>(a.dz_ws + off) = make_float4(dzv[0], dzv[1], dzv[2], dzv[3]);
                    else
                        for (int j = 0; j < 4 && c + j < n; ++j) a.dz_ws[off + j] = dzv[j];
                }
            }
        }
    }
    RT_PP_MARK(0)
    if (prim && a.dbias && a.dbias_slots) {
        // dbias partials: this block's column sums of dz into fp64 slot bid % SLOTS
        // (the dW launch folds the slots; contention per address = blocks / SLOTS)
        __syncthreads();
        double* sl = a.dbias_slots + static_cast<int64_t>(bid % RT_STAT_SLOTS) * n;
        for (int c = tid; c < n; c += 256) {
            float cs = 0.f;
#pragma unroll 8
            for (int r = 0; r < FM; ++r) cs += Dz[r * ldz + c];
            atomicAdd(&sl[c], static_cast<double>(cs));
        }
    }
    if (prim && bid == 0 && (a.grad_mode == 1 || a.grad_mode == 2) && a.dgamma) {
        // dgamma/dbeta of each BN batch (segment), summed like two tower calls' grads
        for (int c = tid; c < n; c += 256) {
            for (int sg = 0; sg < (two ? 2 : 1); ++sg) {
                const double* gs = a.g_stats + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * n;
                double gs1, gs2;
                slot_sums(gs, n, c, gs1, gs2);
                atomicAdd(&a.dgamma[c], static_cast<float>(gs2));  // atomic: concurrent chains of one tower
                atomicAdd(&a.dbeta[c], static_cast<float>(gs1));
            }
        }
    }
    if (!a.g_prev && !a.dsrc) {
#ifndef RT_FOLD_FIRST
        fold_side(L, 0);
#endif
        RT_PP_END(2)
        return;
    }
    __syncthreads();
    RT_PP_MARK(1)

    // ---- phase B: dA = dz · W on the bf16 MFMA (three-piece split) ----
    // the dz tile's pieces go to LDS once per block ([3][FM][ldb] bf16, rows
    // padded by 16 B: the 32 rows of a ds_read_b128 cover the 64 banks); W's
    // are split in registers per k-block
    const int ldb = np + 8;
    uint16_t* const planes = reinterpret_cast<uint16_t*>(Dz + FM * ldz + 5 * np);
    const int plane = FM * ldb;
    for (int e = tid; e < FM * (np / 4); e += 256) {
        const int r = e / (np / 4), c = (e - r * (np / 4)) * 4;
        const float4 v = *reinterpret_cast<const float4*>(Dz + r * ldz + c);
        uint32_t h0, m0, l0, h1, m1, l1;
        split3(v.x, v.y, h0, m0, l0);
        split3(v.z, v.w, h1, m1, l1);
        uint16_t* q = planes + r * ldb + c;
        *reinterpret_cast<uint2*>(q) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(q + plane) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(q + 2 * plane) = make_uint2(l0, l1);
    }
    __syncthreads();
    f32x16 acc[TPWK];
#pragma unroll
    for (int i = 0; i < TPWK; ++i) acc[i] = f32x16{};
    const uint16_t* ap = planes + c32 * ldb + 8 * h;
    const bool want_stats = a.g_prev && a.g_prev_stats && (a.prev_mode == 1 || a.prev_mode == 2);
    // fast epilogue (the C2 hidden layers): a full row block, g_prev only, a
    // piecewise-linear previous activation — no per-element predicates, 32-bit
    // offsets from one base pointer; its z_prev / BN loads are issued HERE,
    // ahead of the reduction, so they land during the MFMAs
    const bool fast = row0 + FM <= m && !a.dsrc && a.g_prev && act_is_piecewise_linear(a.prev_act);
    float zpre[TPWK][16], pmean[TPWK], pinv[TPWK];
#pragma unroll
    for (int i = 0; i < TPWK; ++i) {
        const int kk = (tb + w + 4 * i) * 32 + c32;
        const bool ld = fast && want_stats && kk < k;
        pmean[i] = ld ? a.prev_mean[my_seg * k + kk] : 0.f;
        pinv[i] = ld ? a.prev_invstd[my_seg * k + kk] : 0.f;
        const float* zp = a.src + (row0 + 4 * h) * a.ld_src + kk;
#pragma unroll
        for (int r = 0; r < 16; ++r) zpre[i][r] = ld ? zp[((r & 3) + 8 * (r >> 2)) * a.ld_src] : 0.f;
    }
    if constexpr (WPL) {
        if constexpr (TPWK != 1) load_p(0, pn);
        for (int s = 0; s < np; s += 16) {
#pragma unroll
            for (int i = 0; i < TPWK; ++i)
#pragma unroll
                for (int p = 0; p < 3; ++p) pv[i][p] = pn[i][p];
            if (s + 16 < np) load_p(s + 16, pn);
            Pieces pa;
            pa.hi = *reinterpret_cast<const s16x8*>(ap + s);
            pa.mid = *reinterpret_cast<const s16x8*>(ap + plane + s);
            pa.lo = *reinterpret_cast<const s16x8*>(ap + 2 * plane + s);
#pragma unroll
            for (int i = 0; i < TPWK; ++i) {
                if ((tb + w + 4 * i) * 32 >= k) continue;  // wave-uniform
                const Pieces pb{__builtin_bit_cast(s16x8, pv[i][0]), __builtin_bit_cast(s16x8, pv[i][1]),
                                __builtin_bit_cast(s16x8, pv[i][2])};
                acc[i] = mfma3(pa, pb, acc[i]);
            }
        }
    } else {
    if constexpr (TPWK != 1) load_w(0, wn);
    for (int s = 0; s < np; s += 16) {
#pragma unroll
        for (int i = 0; i < TPWK; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) wv[i][j] = wn[i][j];
        if (s + 16 < np) load_w(s + 16, wn);
        Pieces pa;
        pa.hi = *reinterpret_cast<const s16x8*>(ap + s);
        pa.mid = *reinterpret_cast<const s16x8*>(ap + plane + s);
        pa.lo = *reinterpret_cast<const s16x8*>(ap + 2 * plane + s);
#pragma unroll
        for (int i = 0; i < TPWK; ++i) {
            if ((tb + w + 4 * i) * 32 >= k) continue;  // wave-uniform
            acc[i] = mfma3(pa, split8(wv[i]), acc[i]);
        }
    }
    }
    RT_PP_MARK(2)
    const float pscale = a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f;
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    double* const gps = want_stats ? a.g_prev_stats + (static_cast<int64_t>(my_seg) * RT_STAT_SLOTS +
                                                        bid % RT_STAT_SLOTS) * 2 * k : nullptr;
    const float psl = act_slope(a.prev_act);
#pragma unroll
    for (int i = 0; i < TPWK; ++i) {
        const int kk = (tb + w + 4 * i) * 32 + c32;
        const bool col_ok = kk < k;
        float s1 = 0.f, s2 = 0.f;
        if ((tb + w + 4 * i) * 32 >= k) continue;  // wave-uniform: tile past k
        if (fast) {
            const int64_t rb = row0 + 4 * h;
            float* gp = a.g_prev + rb * k + kk;
            const float* zv = zpre[i];
            const float pm = pmean[i], pi = pinv[i];
            const bool drop = a.prev_drop_p > 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2);
                float gv = acc[i][r];
                if (drop) gv = dropout_keep(pseed, rb + lr, kk, a.prev_drop_p) ? gv * pscale : 0.f;
                if (col_ok) st_act(gp + lr * k, gv);
                const float xh = (act_pwl(psl, zv[r]) - pm) * pi;
                s1 += gv;
                s2 += gv * xh;
            }
            if (!want_stats || !col_ok) s1 = s2 = 0.f;
        } else
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t gr = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (gr < m && col_ok) {
                const float da = acc[i][r];
                if (a.dsrc) a.dsrc[gr * k + kk] = da;
                if (a.g_prev) {
                    float gv = da;
                    if (a.prev_drop_p > 0.f)
                        gv = dropout_keep(pseed, gr, kk, a.prev_drop_p) ? da * pscale : 0.f;
                    a.g_prev[gr * k + kk] = gv;
                    if (want_stats) {
                        const float xh = (act_eval(a.prev_act, a.src[gr * a.ld_src + kk]) -
                                          a.prev_mean[my_seg * k + kk]) * a.prev_invstd[my_seg * k + kk];
                        s1 += gv;
                        s2 += gv * xh;
                    }
                }
            }
        }
        if (want_stats) {
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (h == 0 && col_ok) {
                atomicAdd(&gps[kk], static_cast<double>(s1));
                atomicAdd(&gps[k + kk], static_cast<double>(s2));
            }
        }
    }
#ifndef RT_FOLD_FIRST
    fold_side(L, 0);
#endif
    RT_PP_END(2)
}

// ---------------------------------------------------------------------------
// backward 2: dW[n][k] += Σ_r dz[r][n] · A[r][k] (+ dbias[n] += Σ_r dz[r][n]),
// M split over the blocks of a group
// ---------------------------------------------------------------------------
// Block = one BN(n) x BK(k) tile of dW over a contiguous row range, 8 waves in
// two row groups of 4 (each group's waves own the tile's 32x32 sub-tiles; the
// groups take alternate row pairs and are summed through LDS at the end).
// Rows stream in 32-row chunks staged ROW-MAJOR in LDS (float4 loads → one
// ds_write_b128, no transposition), double-buffered: chunk c+1's global loads
// are in flight during chunk c's MFMAs and land in the other buffer. The MFMA
// operands are read straight from the row-major tiles: for the row pair
// (2p, 2p+1) lane c of half h reads dz[2p+h][n-col c] and A[2p+h][k-col c]
// (ds_read_b32; row strides ≡ 32 mod 64 banks, so the halves never collide),
// i.e. v_mfma_f32_32x32x2_f32 with the row pair as its k = 2. A goes through
// the forward's own prologue (act → BN affine → dropout) while it is staged.
// The tile is added to dW with one fp32 atomic per element per block (one
// 128-B row segment per lane half); blocks of k-tile 0 also add dbias.
//   PRO: 0 raw A, 1 piecewise-linear act, 2 same + dropout, 3 generic act.
constexpr int DW_R = 32;          // rows per chunk
constexpr int DW_G = 2;           // row groups (waves 4g..4g+3)
constexpr int DW_NT = 256 * DW_G; // threads per block
constexpr int DW_MAXR = 2048;     // rows per split whose gather ids are staged in LDS

__host__ __device__ constexpr int dw_ld(int x) { return x + ((x / 32) % 2 == 0 ? 32 : 0); }  // ≡ 32 mod 64

template <int PRO>
__device__ __forceinline__ float pro_col(const Pro& p, float slope, int64_t r, int c, float sc, float sh, float v) {
    if constexpr (PRO == 0) {
        return v;
    } else {
        if constexpr (PRO == 3) v = act_eval(p.act, v);
        else v = act_pwl(slope, v);
        v = __builtin_fmaf(v, sc, sh);
        if constexpr (PRO == 2) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
        if constexpr (PRO == 3) {
            if (p.drop_p > 0.f) v = dropout_keep(p.seed, r, c, p.drop_p) ? v * p.drop_scale : 0.f;
        }
        return v;
    }
}

// DZF: the layer has no dA (the first Linear of a chain); the dz launch was
// skipped (rt_linear_bwd_args.fuse_dz) and dz is computed here while staged,
// from g and z with the per-column BN-backward coefficients, exactly as the dz
// launch's phase A would; dgamma/dbeta (block 0) and dbias (row sums of the
// computed dz) are added here too.
template <int BN, int BK, int PRO, bool VEC, bool DZF>  // VEC: n, k, ld_src multiples of 4, 16-B aligned rows
__global__ __launch_bounds__(DW_NT) void linear_bwd_dw_kernel(BwdLaunch L) {
    constexpr int NTN = BN / 32, WK = 4 / NTN, T = (BK / 32) / WK;
    static_assert(NTN * 32 == BN && 4 % NTN == 0 && T >= 1 && T * WK * 32 == BK, "dW tile");
    constexpr int LDN = dw_ld(BN), LDK = dw_ld(BK);
    constexpr int VN = BN / 4, VK = BK / 4;  // float4 per row
    constexpr int LN = (DW_R * VN + DW_NT - 1) / DW_NT, LK = (DW_R * VK + DW_NT - 1) / DW_NT;
    static_assert(DW_NT % VN == 0 && DW_NT % VK == 0, "fixed staging columns per thread");
    static_assert(2 * DW_R * LDN >= 4 * T * 16 * 64, "row-group reduction fits in the dz buffers");
    static_assert(2 * DW_R * LDK >= (DW_NT / 64) * VN * 4, "dbias partials fit in the A buffers");
    __shared__ __attribute__((aligned(16))) float Ld[2][DW_R * LDN];
    __shared__ __attribute__((aligned(16))) float La[2][DW_R * LDK];
    // gather ids staged for the first Linear only (PRO 0): the other instances
    // stay at <= 53 KB of LDS, 3 blocks per CU (the C2 layer-2 dW launch's ~750
    // blocks then run as one wave of blocks instead of two)
    __shared__ int srow[PRO == 0 ? DW_MAXR : 1];
    __shared__ __attribute__((aligned(16))) float aff_s[2][2][BK];  // [segment][scale, shift][tile column]
    __shared__ __attribute__((aligned(16))) float dzc_s[DZF ? 2 : 1][5][DZF ? BN : 4];  // DZF: [seg][A,B,C,M,I][col]

#ifdef RT_FOLD_FIRST
    fold_side(L, 1);
#endif
    const bool g1 = blockIdx.x >= L.split;
    const rt_linear_bwd_args a = g1 ? L.a1 : L.a0;  // by value: fields loaded once
    const int64_t rows_per_split = g1 ? L.rps1 : L.rps0;
    const unsigned bid = blockIdx.x - (g1 ? L.split : 0u);
    const unsigned tn = g1 ? L.tn1 : L.tn0, tk = g1 ? L.tk1 : L.tk0;
    const unsigned bx = bid % tn, by = (bid / tn) % tk, bz = bid / (tn * tk);
    const int n = a.n, k = a.k;
    const int64_t m = a.m;
    const int tid = threadIdx.x, lane = tid & 63, wg = tid >> 6, w = wg & 3, grp = wg >> 2, h = lane >> 5,
              c = lane & 31;
    const int n0 = static_cast<int>(bx) * BN, k0 = static_cast<int>(by) * BK;
    const int64_t r_begin = static_cast<int64_t>(bz) * rows_per_split;
    const int64_t r_end = (r_begin + rows_per_split) < m ? (r_begin + rows_per_split) : m;
    if (r_begin >= m) {  // a padding split (block-uniform, before any barrier)
#ifndef RT_FOLD_FIRST
        fold_side(L, 1);
#endif
        return;
    }
    RT_PP_DECL
    // A rows: the forward's staged copy (a_in, read as is: PRO 0) or recomputed from src
    const bool gather = PRO == 0 && a.ids != nullptr && !a.a_in;  // (the host refuses ids with a transformed input)
    const float* const asrc = a.a_in ? a.a_in : a.src;
    const int64_t ald = a.a_in ? static_cast<int64_t>(k) : static_cast<int64_t>(a.ld_src);
    const bool two = a.seg_split > 0;

    // staging columns of this thread (the same for every staged row)
    const int cn = (tid % VN) * 4, ck = (tid % VK) * 4;
    const int gn = n0 + cn, gk = k0 + ck;
    // BN affine of the previous block for this thread's 4 A columns, per row segment
    float4 sc0 = make_float4(1.f, 1.f, 1.f, 1.f), sc1 = sc0;
    float4 sh0 = make_float4(0.f, 0.f, 0.f, 0.f), sh1 = sh0;
    if ((a.prev_mode == 1 || a.prev_mode == 2) && !a.a_in) {
        // one load per (segment, column) for the whole block, through LDS: with
        // every thread loading its own 4 columns x 2 segments x 4 arrays, the
        // 512 threads x ~750 blocks of a C2 launch hammered the same few L2
        // lines (7.4 us of prologue per block, tools/c2_phase_probe.py)
        if (tid < 2 * BK) {
            const int sg = tid / BK, cl = tid % BK, cc = k0 + cl;
            const int so = two ? sg * k : 0;
            float scv = 1.f, shv = 0.f;
            if (cc < k) bn_affine(a.prev_gamma[cc], a.prev_beta[cc], a.prev_mean[so + cc], a.prev_invstd[so + cc], scv, shv);
            aff_s[sg][0][cl] = scv;
            aff_s[sg][1][cl] = shv;
        }
        __syncthreads();
        sc0 = *reinterpret_cast<const float4*>(&aff_s[0][0][ck]);
        sh0 = *reinterpret_cast<const float4*>(&aff_s[0][1][ck]);
        sc1 = *reinterpret_cast<const float4*>(&aff_s[1][0][ck]);
        sh1 = *reinterpret_cast<const float4*>(&aff_s[1][1][ck]);
    }
    const uint64_t pseed = a.prev_drop_seed + (a.seed_offset ? *a.seed_offset : 0ull);
    const Pro pro{a.prev_mode, a.prev_act, a.prev_drop_p, a.prev_drop_p > 0.f ? 1.f / (1.f - a.prev_drop_p) : 1.f,
                  pseed, nullptr, nullptr};
    const float slope = act_slope(a.prev_act);
    if constexpr (DZF) {
        // per-column BN-backward coefficients of this block's n-tile, per row
        // segment (the dz launch's phase A): A = γ·invstd (or 1), B = Σg/m,
        // C = Σg·x̂/m, M = mean, I = invstd
        if (tid < 2 * BN) {
            const int sg = tid / BN, cl = tid % BN, c = n0 + cl;
            const int my = two ? sg : 0;
            const int64_t seg_m = two ? (my == 0 ? a.seg_split : m - a.seg_split) : m;
            float A = 1.f, Bc = 0.f, C = 0.f, M = 0.f, I = 1.f;
            if (c < n && (a.grad_mode == 1 || a.grad_mode == 2)) {
                I = a.save_invstd[my * n + c];
                M = a.save_mean[my * n + c];
                A = a.bn_gamma[c] * I;
                if (a.grad_mode == 1) {
                    double gs1, gs2;
                    slot_sums(a.g_stats + static_cast<int64_t>(my) * RT_STAT_SLOTS * 2 * n, n, c, gs1, gs2);
                    const float inv_m = 1.f / static_cast<float>(seg_m);
                    Bc = static_cast<float>(gs1) * inv_m;
                    C = static_cast<float>(gs2) * inv_m;
                }
            }
            dzc_s[sg][0][cl] = A; dzc_s[sg][1][cl] = Bc; dzc_s[sg][2][cl] = C;
            dzc_s[sg][3][cl] = M; dzc_s[sg][4][cl] = I;
        }
        if (bid == 0 && (a.grad_mode == 1 || a.grad_mode == 2) && a.dgamma) {
            // dgamma/dbeta of each BN batch (segment), as the dz launch's block 0
            for (int c = tid; c < n; c += DW_NT) {
                for (int sg = 0; sg < (two ? 2 : 1); ++sg) {
                    double gs1, gs2;
                    slot_sums(a.g_stats + static_cast<int64_t>(sg) * RT_STAT_SLOTS * 2 * n, n, c, gs1, gs2);
                    atomicAdd(&a.dgamma[c], static_cast<float>(gs2));
                    atomicAdd(&a.dbeta[c], static_cast<float>(gs1));
                }
            }
        }
        __syncthreads();
    }
    // dbias: folded from the dz launch's fp64 slots by block 0, or (no slots,
    // or dz computed here) summed here by the k-tile-0 blocks
    if (!DZF && a.dbias && a.dbias_slots && bid == 0) {
        for (int cc = tid; cc < n; cc += DW_NT) {
            double v = 0.0;
#pragma unroll
            for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) v += a.dbias_slots[static_cast<int64_t>(sl) * n + cc];
            atomicAdd(&a.dbias[cc], static_cast<float>(v));
        }
    }
    const bool do_bias = a.dbias != nullptr && (DZF || a.dbias_slots == nullptr) && by == 0;
    // fused dz with slots: same-address fp32 dbias atomics from every split of a
    // tile cost ~10 us per C2 step (a timing build without them); instead the
    // splits add into the fp64 slots and the tile's last-arriving block folds
    // them (ticket counter in slot row RT_STAT_SLOTS, zeroed with the slots)
    const bool slot_bias = DZF && do_bias && a.dbias_slots != nullptr;

    if (gather) {
        for (int64_t t = tid; t < r_end - r_begin; t += DW_NT) {
            const int64_t id = a.ids[r_begin + t];
            srow[t] = (id < 0 || id >= a.src_rows) ? -1 : static_cast<int>(id);
        }
        __syncthreads();
    }

    float4 rd[LN], rz[DZF ? LN : 1], ra[LK];  // one chunk's staged values (prefetch registers)
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    const float dsl = act_slope(a.act);
    auto load = [&](int64_t base) {
#pragma unroll
        for (int j = 0; j < LN; ++j) {
            const int e = tid + DW_NT * j, row = e / VN;
            const int64_t r = base + row;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (DZF) {  // g and z of the row (n % 4 == 0, checked by the host)
                float4 zv = v;
                if (e < DW_R * VN && r < r_end && gn < n) {
                    v = *reinterpret_cast<const float4*>(a.g + r * n + gn);
                    zv = *reinterpret_cast<const float4*>(a.z + r * n + gn);
                }
                rd[j] = v;
                rz[j] = zv;
                continue;
            }
            if (e < DW_R * VN && r < r_end) {
                const float* dz = a.dz_ws + r * n + gn;
                if constexpr (VEC) {
                    if (gn < n) v = *reinterpret_cast<const float4*>(dz);
                } else {
                    if (gn < n) v.x = dz[0];
                    if (gn + 1 < n) v.y = dz[1];
                    if (gn + 2 < n) v.z = dz[2];
                    if (gn + 3 < n) v.w = dz[3];
                }
            }
            rd[j] = v;
        }
#pragma unroll
        for (int j = 0; j < LK; ++j) {
            const int e = tid + DW_NT * j, row = e / VK;
            const int64_t r = base + row;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < DW_R * VK && r < r_end) {
                const int64_t sr = gather ? srow[r - r_begin] : r;
                if (sr >= 0) {
                    const float* ap = asrc + sr * ald + gk;
                    if constexpr (VEC) {
                        if (gk < k) v = *reinterpret_cast<const float4*>(ap);
                    } else {
                        if (gk < k) v.x = ap[0];
                        if (gk + 1 < k) v.y = ap[1];
                        if (gk + 2 < k) v.z = ap[2];
                        if (gk + 3 < k) v.w = ap[3];
                    }
                }
            }
            ra[j] = v;
        }
    };
    auto store = [&](int buf, int64_t base) {
#pragma unroll
        for (int j = 0; j < LN; ++j) {
            const int e = tid + DW_NT * j, row = e / VN;
            if (e < DW_R * VN) {
                if constexpr (DZF) {
                    // dz = A·(g − B − x̂·C)·act'(z), x̂ = (act(z) − M)·I (phase A of the dz launch)
                    const int64_t r = base + row;
                    const int sg = (two && r >= a.seg_split) ? 1 : 0;
                    const bool ok = r < r_end;
                    float4 d;
                    auto one = [&](float g, float z, int i) {
                        const int cl = cn + i;
                        const float A = dzc_s[sg][0][cl], Bc = dzc_s[sg][1][cl], C = dzc_s[sg][2][cl];
                        const float M = dzc_s[sg][3][cl], I = dzc_s[sg][4][cl];
                        const float xh = (act_pwl(dsl, z) - M) * I;
                        return (ok && gn + i < n) ? A * (g - Bc - xh * C) * (z > 0.f ? 1.f : dsl) : 0.f;
                    };
                    d.x = one(rd[j].x, rz[j].x, 0);
                    d.y = one(rd[j].y, rz[j].y, 1);
                    d.z = one(rd[j].z, rz[j].z, 2);
                    d.w = one(rd[j].w, rz[j].w, 3);
                    rd[j] = d;
                }
                *reinterpret_cast<float4*>(&Ld[buf][row * LDN + cn]) = rd[j];
                bsum.x += rd[j].x; bsum.y += rd[j].y; bsum.z += rd[j].z; bsum.w += rd[j].w;
            }
        }
#pragma unroll
        for (int j = 0; j < LK; ++j) {
            const int e = tid + DW_NT * j, row = e / VK;
            if (e < DW_R * VK) {
                const int64_t r = base + row;
                const bool ok = r < r_end && (!gather || srow[r - r_begin] >= 0);
                const bool hi_seg = two && r >= a.seg_split;
                const float4 scs = hi_seg ? sc1 : sc0, shs = hi_seg ? sh1 : sh0;
                float4 v;
                v.x = (ok && gk < k) ? pro_col<PRO>(pro, slope, r, gk, scs.x, shs.x, ra[j].x) : 0.f;
                v.y = (ok && gk + 1 < k) ? pro_col<PRO>(pro, slope, r, gk + 1, scs.y, shs.y, ra[j].y) : 0.f;
                v.z = (ok && gk + 2 < k) ? pro_col<PRO>(pro, slope, r, gk + 2, scs.z, shs.z, ra[j].z) : 0.f;
                v.w = (ok && gk + 3 < k) ? pro_col<PRO>(pro, slope, r, gk + 3, scs.w, shs.w, ra[j].w) : 0.f;
                *reinterpret_cast<float4*>(&La[buf][row * LDK + ck]) = v;
            }
        }
    };

    f32x16 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = f32x16{};
    const int ncol = (w % NTN) * 32 + c;       // this lane's dz column inside the tile
    const int kcol0 = (w / NTN) * T * 32 + c;  // this lane's first A column inside the tile
    int buf = 0;
    RT_PP_MARK(0)
    load(r_begin);
    store(0, r_begin);
    __syncthreads();
    RT_PP_MARK(1)
    for (int64_t base = r_begin; base < r_end; base += DW_R) {
        const bool more = base + DW_R < r_end;  // block-uniform
        if (more) load(base + DW_R);            // in flight during the MFMAs below
        // row pairs grp, grp + DW_G, ...: lane half h reads row 2·pair + h
        const float* dl = &Ld[buf][(2 * grp + h) * LDN + ncol];
        const float* al = &La[buf][(2 * grp + h) * LDK + kcol0];
#pragma unroll
        for (int i = 0; i < DW_R / (2 * DW_G); ++i) {
            const float av = dl[2 * DW_G * i * LDN];
#pragma unroll
            for (int t = 0; t < T; ++t) acc[t] = mfma(av, al[2 * DW_G * i * LDK + 32 * t], acc[t]);
        }
        if (more) store(buf ^ 1, base + DW_R);
        __syncthreads();
        buf ^= 1;
    }

    // dbias: column sums of dz over this block's rows. Threads sharing the
    // staging columns cn (lanes l ^ 16·j when VN = 16, l ^ 32 when VN = 32) are
    // summed by shuffles, the 8 waves through LDS, then ONE atomic per column
    // per block (same-address float atomics serialise: 8 per block measured
    // 40-80 µs at the C2 shapes). Each row group adds half of the dW tile and
    // hands the other half of its accumulators to the other group through the
    // (idle) dz buffers (both groups issue atomics: 1.5 µs/step faster than
    // group 0 adding all of it); the dbias partials go through the A buffers.
    RT_PP_MARK(2)
    float* red = &Ld[0][0];
    float* bred = &La[0][0];  // [8 waves][VN][4]
    if (do_bias) {
#pragma unroll
        for (int o = VN; o < 64; o <<= 1) {
            bsum.x += __shfl_xor(bsum.x, o, 64);
            bsum.y += __shfl_xor(bsum.y, o, 64);
            bsum.z += __shfl_xor(bsum.z, o, 64);
            bsum.w += __shfl_xor(bsum.w, o, 64);
        }
        if (lane < VN) *reinterpret_cast<float4*>(&bred[(wg * VN + lane) * 4]) = bsum;
    }
    // row group grp adds accumulator rows 8·grp .. 8·grp+7 of the tile
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if ((r >> 3) != grp) red[((w * T + t) * 16 + r) * 64 + lane] = acc[t][r];
    __syncthreads();
    if (do_bias && tid < VN) {
        float4 sb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int o = 0; o < DW_NT / 64; ++o) {
            const float4 v = *reinterpret_cast<const float4*>(&bred[(o * VN + tid) * 4]);
            sb.x += v.x; sb.y += v.y; sb.z += v.z; sb.w += v.w;
        }
        const int cb = n0 + tid * 4;
        if (slot_bias) {
            // fused-dz launch: the split's column sums go to fp64 slot bz % SLOTS
            // (contention splits / SLOTS per address instead of splits); the
            // tile's last block folds the slots below
            double* sl = a.dbias_slots + static_cast<int64_t>(bz % RT_STAT_SLOTS) * n;
            if (cb < n) atomicAdd(&sl[cb], static_cast<double>(sb.x));
            if (cb + 1 < n) atomicAdd(&sl[cb + 1], static_cast<double>(sb.y));
            if (cb + 2 < n) atomicAdd(&sl[cb + 2], static_cast<double>(sb.z));
            if (cb + 3 < n) atomicAdd(&sl[cb + 3], static_cast<double>(sb.w));
        } else {
            if (cb < n) atomicAdd(&a.dbias[cb], sb.x);
            if (cb + 1 < n) atomicAdd(&a.dbias[cb + 1], sb.y);
            if (cb + 2 < n) atomicAdd(&a.dbias[cb + 2], sb.z);
            if (cb + 3 < n) atomicAdd(&a.dbias[cb + 3], sb.w);
        }
    }
    // acc[t][r] = dW[n0 + ncol-tile + (r&3) + 8(r>>2) + 4h][k0 + kcol0 + 32t]
    auto add_row = [&](int t, int r, int kk) {
        const int nn = n0 + (w % NTN) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = acc[t][r] + red[((w * T + t) * 16 + r) * 64 + lane];
        if (nn < n) {
            if (a.dw_part) {  // folded by a later launch; write-through (1 us/step better than plain)
#ifdef RT_DW_PART_PLAIN
                a.dw_part[(static_cast<int64_t>(bz) * n + nn) * k + kk] = v;
#else
                st_act(a.dw_part + (static_cast<int64_t>(bz) * n + nn) * k + kk, v);
#endif
            }
            else atomicAdd(&a.dw[static_cast<int64_t>(nn) * k + kk], v);
        }
    };
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int kk = k0 + kcol0 + 32 * t;
        if (kk >= k) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if ((r >> 3) == grp) add_row(t, r, kk);
    }
    if (slot_bias) {  // block-uniform
        __shared__ int last_s;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slot atomics are performed
        __syncthreads();
        if (tid == 0) {
            ticket_release();
            unsigned long long* cnt = reinterpret_cast<unsigned long long*>(a.dbias_slots + static_cast<int64_t>(RT_STAT_SLOTS) * n);
            const unsigned long long nsplit = static_cast<unsigned long long>((m + rows_per_split - 1) / rows_per_split);
            last_s = atomicAdd(&cnt[bx], 1ull) == nsplit - 1 ? 1 : 0;
        }
        __syncthreads();
        if (last_s) {
            // every split of this tile has added: fold the slots in slot order
            // (returning adds of 0 read them at the memory side, where they live)
            for (int cl = tid; cl < BN; cl += DW_NT) {
                const int c = n0 + cl;
                if (c >= n) continue;
                double v = 0.0;
#pragma unroll
                for (int sl = 0; sl < RT_STAT_SLOTS; ++sl) v += atomicAdd(&a.dbias_slots[static_cast<int64_t>(sl) * n + c], 0.0);
                atomicAdd(&a.dbias[c], static_cast<float>(v));
            }
        }
    }
#ifndef RT_FOLD_FIRST
    fold_side(L, 1);
#endif
    RT_PP_END(3)
}

}  // namespace mlp
}  // namespace rt

using namespace rt;

// allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); set once per kernel
template <typename K>
static void allow_lds(K kernel, size_t bytes) {
    static size_t set = 0;
    if (bytes > set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(bytes));
        set = bytes;
    }
}

static int validate_fwd(const rt_linear_fwd_args* args) {
    if (!args) return RT_ERR_INVALID;
    const rt_linear_fwd_args& a = *args;
    if (a.m < 0 || a.k <= 0 || a.n <= 0 || !a.src || !a.w || a.ld_src < a.k) return RT_ERR_INVALID;
    if (a.n > 512 || a.k > 8192) return RT_ERR_UNSUPPORTED;
    if (a.prev_mode < 0 || a.prev_mode > 3) return RT_ERR_INVALID;
    if (a.seg_split < 0 || (a.seg_split > 0 && (a.seg_split >= a.m || a.seg_split % mlp::FM != 0)))
        return RT_ERR_INVALID;
    if (a.prev_mode == 1 && (!a.prev_stats || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.prev_mode == 2 && (!a.running_mean || !a.running_var || !a.bn_gamma || !a.bn_beta)) return RT_ERR_INVALID;
    if (a.a_out && ((a.k % 4) != 0 || (reinterpret_cast<uintptr_t>(a.a_out) & 15) != 0)) return RT_ERR_INVALID;
    if (a.fin_save_mean && (!a.stats_out || !a.fin_save_invstd || (!a.fin_running_mean != !a.fin_running_var)))
        return RT_ERR_INVALID;
    if (a.prev_final && (a.prev_mode != 1 || !a.save_mean || !a.save_invstd)) return RT_ERR_INVALID;
    if (a.w_planes && ((a.k % 8) != 0 || a.n > 128 || (reinterpret_cast<uintptr_t>(a.w_planes) & 15) ||
                       (reinterpret_cast<uintptr_t>(a.w) & 15)))
        return RT_ERR_INVALID;
    if (a.next_w_planes && (!a.next_w || a.next_n <= 0 || a.next_k <= 0 || (a.next_k % 8) != 0 ||
                            (reinterpret_cast<uintptr_t>(a.next_w) & 15) ||
                            (reinterpret_cast<uintptr_t>(a.next_w_planes) & 15)))
        return RT_ERR_INVALID;
    const int kp = mlp::pad8(a.k);
    const int tpw = a.n <= 128 ? 1 : a.n <= 256 ? 2 : 4;
    const size_t lds = (2 * kp + 3 * mlp::FM * kp / 2 + 4 * tpw * mlp::FM) * sizeof(float) + mlp::FM * sizeof(int64_t) + 16;
    if (lds > 160 * 1024) return RT_ERR_UNSUPPORTED;
    return RT_OK;
}

extern "C" int rt_linear_fwd_f32_multi(const rt_linear_fwd_args* args, int n_args, void* stream) {
    if (!args || n_args < 1 || n_args > 2) return RT_ERR_INVALID;
#ifdef RT_NO_AIN  // A/B build: no staged-input copy (the dW launch recomputes A)
    rt_linear_fwd_args noa[2];
    for (int g = 0; g < n_args; ++g) { noa[g] = args[g]; noa[g].a_out = nullptr; }
    args = noa;
#endif
    int tpw = 1, kp_max = 0;
    bool kvec = true, wpl = true;  // wpl: every argument set brings its W planes
    unsigned blocks[2] = {0u, 0u};
    for (int g = 0; g < n_args; ++g) {
        const int v = validate_fwd(&args[g]);
        if (v) return v;
        const rt_linear_fwd_args& a = args[g];
        wpl = wpl && a.w_planes != nullptr;
        const int t = a.n <= 128 ? 1 : a.n <= 256 ? 2 : 4;
        tpw = t > tpw ? t : tpw;
        kvec = kvec && (a.k % 4) == 0 && (reinterpret_cast<uintptr_t>(a.w) & 15) == 0;
        const int kp = mlp::pad8(a.k);
        kp_max = kp > kp_max ? kp : kp_max;
        blocks[g] = static_cast<unsigned>((a.m + mlp::FM - 1) / mlp::FM);
    }
    // LDS carve-up of the kernel built for tpw tiles at the larger k of the two
    const size_t lds = (2 * kp_max + 3 * mlp::FM * kp_max / 2 + 4 * tpw * mlp::FM) * sizeof(float) +
                       mlp::FM * sizeof(int64_t) + 16;
    if (lds > 160 * 1024) return RT_ERR_UNSUPPORTED;
    mlp::FwdLaunch L{};
    L.a0 = args[0];
    L.a1 = n_args > 1 ? args[1] : args[0];
    L.split = blocks[0];
    const unsigned total = blocks[0] + (n_args > 1 ? blocks[1] : 0u);
    if (total == 0) return RT_OK;
    hipStream_t st = as_stream(stream);
    const dim3 grid(total);
#define RT_FWD(T, V, P)                                                                           \
    do {                                                                                          \
        allow_lds(mlp::linear_fwd_kernel<T, V, P>, lds);                                          \
        hipLaunchKernelGGL((mlp::linear_fwd_kernel<T, V, P>), grid, dim3(256), lds, st, L);       \
    } while (0)
    if (kvec && tpw == 1 && wpl) {
        RT_FWD(1, true, true);
    } else if (kvec) {
        if (tpw == 1) RT_FWD(1, true, false); else if (tpw == 2) RT_FWD(2, true, false); else RT_FWD(4, true, false);
    } else {
        if (tpw == 1) RT_FWD(1, false, false); else if (tpw == 2) RT_FWD(2, false, false); else RT_FWD(4, false, false);
    }
#undef RT_FWD
    return check_launch("linear_fwd_kernel");
}

extern "C" int rt_linear_fwd_f32(const rt_linear_fwd_args* args, void* stream) {
    return rt_linear_fwd_f32_multi(args, 1, stream);
}

// the dz launch of a dA-free layer (first Linear, no input gradient) folds into
// its dW launch (rt_linear_bwd_args.fuse_dz): piecewise-linear activation,
// BN modes 1-3, n % 4 == 0
static bool dz_fusable(const rt_linear_bwd_args& a) {
#ifdef RT_NO_DZ_FUSE  // A/B variant: always the separate dz launch
    return false;
#endif
    return a.fuse_dz && !a.g_prev && !a.dsrc && a.grad_mode >= 1 && a.grad_mode <= 3 &&
           act_is_piecewise_linear(a.act) && (a.n % 4) == 0 && a.g && a.z &&
           (reinterpret_cast<uintptr_t>(a.g) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.z) & 15) == 0;
}
static bool all_dz_fusable(const rt_linear_bwd_args* args, int n_args) {
    for (int g = 0; g < n_args; ++g)
        if (!dz_fusable(args[g])) return false;
    return true;
}

static int validate_bwd(const rt_linear_bwd_args* args) {
    if (!args) return RT_ERR_INVALID;
    const rt_linear_bwd_args& a = *args;
    if (a.m < 0 || a.k <= 0 || a.n <= 0 || !a.w || !a.dw || !a.dz_ws || !a.src || a.ld_src < a.k)
        return RT_ERR_INVALID;
    const bool need_da = a.g_prev || a.dsrc;
    if (a.n > 2048 || (need_da && a.k > 512)) return RT_ERR_UNSUPPORTED;
    if (a.grad_mode == 0 && (!a.dout || !a.l2_out || !a.norms)) return RT_ERR_INVALID;
    if (a.grad_mode >= 1 && a.grad_mode <= 3 && (!a.g || !a.z)) return RT_ERR_INVALID;
    if ((a.grad_mode == 1 || a.grad_mode == 2) && (!a.g_stats || !a.save_mean || !a.save_invstd || !a.bn_gamma))
        return RT_ERR_INVALID;
    if (a.grad_mode < 0 || a.grad_mode > 3) return RT_ERR_INVALID;
    if (a.seg_split < 0 || (a.seg_split > 0 && (a.seg_split >= a.m || a.seg_split % mlp::FM != 0)))
        return RT_ERR_INVALID;
    if ((a.prev_mode == 1 || a.prev_mode == 2) &&
        (!a.prev_mean || !a.prev_invstd || !a.prev_gamma || !a.prev_beta))
        return RT_ERR_INVALID;
    if (a.fold_src && (!a.fold_dst || a.fold_words % 4 != 0 || a.fold_splits <= 0 || a.fold_in < 0 || a.fold_in > 1 ||
                       (reinterpret_cast<uintptr_t>(a.fold_src) & 15) || (reinterpret_cast<uintptr_t>(a.fold_dst) & 15)))
        return RT_ERR_INVALID;
    if (a.wt_planes && ((a.n % 8) != 0 || (reinterpret_cast<uintptr_t>(a.wt_planes) & 15))) return RT_ERR_INVALID;
    return RT_OK;
}

extern "C" int rt_linear_bwd_dz_f32_multi(const rt_linear_bwd_args* args, int n_args, void* stream) {
    if (!args || n_args < 1 || n_args > 2) return RT_ERR_INVALID;
    int tpwk = 1;
    size_t lds = 0;
    unsigned blocks[2] = {0u, 0u};
    bool wpl = true;  // every argument set with a dA brings Wᵀ's planes
    for (int g = 0; g < n_args; ++g) {
        const int v = validate_bwd(&args[g]);
        if (v) return v;
        const rt_linear_bwd_args& a = args[g];
        const bool need_da = a.g_prev || a.dsrc;
        wpl = wpl && (!need_da || a.wt_planes != nullptr);
        const int t = !need_da ? 1 : a.k <= 128 ? 1 : a.k <= 256 ? 2 : 4;
        tpwk = t > tpwk ? t : tpwk;
        const int np = mlp::pad8(a.n);
        const size_t l = (static_cast<size_t>(mlp::FM) * (np + 4) + 5 * static_cast<size_t>(np)) * sizeof(float) +
                         3 * static_cast<size_t>(mlp::FM) * (np + 8) * sizeof(uint16_t) + 16;
        lds = l > lds ? l : lds;
        blocks[g] = static_cast<unsigned>((a.m + mlp::FM - 1) / mlp::FM);
    }
    if (all_dz_fusable(args, n_args)) {  // dz computed by the dW launch
        for (int g = 0; g < n_args; ++g)
            if (args[g].fold_src && args[g].fold_in == 0) return RT_ERR_INVALID;  // its fold would never run
        return RT_OK;
    }
    mlp::BwdLaunch L{};
    L.a0 = args[0];
    L.a1 = n_args > 1 ? args[1] : args[0];
    L.ngroups = n_args;
    L.split = blocks[0];
    const unsigned total = blocks[0] + (n_args > 1 ? blocks[1] : 0u);
    if (total == 0) return RT_OK;
    // at most one row block per CU with two dA tiles per wave (the C1
    // dz launch at k = 256: 144 row blocks): each row block's dA columns as
    // two blocks of one tile per wave (RT_DZ_KSPLIT=1/2 forces it, A/B)
    bool any_da = false;
    for (int g = 0; g < n_args; ++g) any_da = any_da || args[g].g_prev || args[g].dsrc;
    static const int ks_env = [] { const char* e = getenv("RT_DZ_KSPLIT"); return e ? atoi(e) : 0; }();
    unsigned ks = (tpwk == 2 && any_da && total <= 256u) ? 2u : 1u;
    if (ks_env == 1 || (ks_env == 2 && tpwk == 2 && any_da)) ks = static_cast<unsigned>(ks_env);
    L.ksplit = ks;
    if (ks == 2) tpwk = 1;
    const dim3 grid(total * ks);
    hipStream_t st = as_stream(stream);
#define RT_DZ(T, P, K)                                                                        \
    do {                                                                                      \
        allow_lds(mlp::linear_bwd_dz_kernel<T, P, K>, lds);                                   \
        hipLaunchKernelGGL((mlp::linear_bwd_dz_kernel<T, P, K>), grid, dim3(256), lds, st, L); \
    } while (0)
    if (ks > 1) {
        if (wpl) RT_DZ(1, true, true); else RT_DZ(1, false, true);
    } else {
        switch (tpwk) {
            case 1: if (wpl) RT_DZ(1, true, false); else RT_DZ(1, false, false); break;
            case 2: if (wpl) RT_DZ(2, true, false); else RT_DZ(2, false, false); break;
            default: RT_DZ(4, false, false); break;
        }
    }
#undef RT_DZ
    return check_launch("linear_bwd_dz_kernel");
}

extern "C" int rt_linear_bwd_dz_fused(const rt_linear_bwd_args* args, int n_args) {
    return (args && n_args >= 1 && n_args <= 2 && all_dz_fusable(args, n_args)) ? 1 : 0;
}

extern "C" int rt_linear_bwd_dz_f32(const rt_linear_bwd_args* args, void* stream) {
    return rt_linear_bwd_dz_f32_multi(args, 1, stream);
}

// dW tiling of one launch (one or two Linears): 64x64 tiles (128x32 when
// k <= 32), whole 32-row chunks, ONE rows-per-split for both groups so that
// every block carries the same work (round 3 split each group for ~512 blocks
// of its own: the user tower's 1,024 rows went out as 32-row blocks that each
// added a whole tile with atomics). About RT_DW_BLOCKS blocks (tiles x row
// splits; each block adds one tile with fp32 atomics, so atomic bytes =
// blocks x tile); <= 64 splits per group (128 when k <= 32); <= DW_MAXR rows
// per split (gather ids staged in LDS). A/B at C2 (profiles/r04_c2_ab_dw_plan.txt):
// 384 / 512 / 768 blocks within 1 µs of each other, 2-2.5 µs/step under the
// per-group plan; an XCD-contiguous block order (the tiles of a split on one
// XCD, sharing its L2) was 7 µs/step SLOWER and is not used.
#ifndef RT_DW_BLOCKS
#define RT_DW_BLOCKS 384
#endif
#ifndef RT_DW_BLOCKS_SMALLK
#define RT_DW_BLOCKS_SMALLK 256
#endif
static void dw_plan(const rt_linear_bwd_args* args, int n_args, bool small_k, unsigned* tn, unsigned* tk,
                    int64_t* splits, int64_t& rps) {
    const int bn = small_k ? 128 : 64, bk = small_k ? 32 : 64;
#ifndef RT_DW_CAP_SMALLK
#define RT_DW_CAP_SMALLK 128
#endif
    const int64_t cap = small_k ? RT_DW_CAP_SMALLK : 64;
    int64_t work = 0, rmin = mlp::DW_R;
    for (int g = 0; g < n_args; ++g) {
        const rt_linear_bwd_args& a = args[g];
        tn[g] = static_cast<unsigned>((a.n + bn - 1) / bn);
        tk[g] = static_cast<unsigned>((a.k + bk - 1) / bk);
        work += a.m * tn[g] * tk[g];
        const int64_t r = (a.m + cap - 1) / cap;
        rmin = r > rmin ? r : rmin;
    }
    const int64_t target = small_k ? RT_DW_BLOCKS_SMALLK : RT_DW_BLOCKS;
    rps = (work + target - 1) / target;
    rps = rps > rmin ? rps : rmin;
    rps = (rps + mlp::DW_R - 1) / mlp::DW_R * mlp::DW_R;
    for (int g = 0; g < n_args; ++g)
        if (args[g].ids && rps > mlp::DW_MAXR) rps = mlp::DW_MAXR;
    for (int g = 0; g < n_args; ++g) splits[g] = args[g].m > 0 ? (args[g].m + rps - 1) / rps : 0;
}

// the dW prologue a set needs: 0 raw input (or the forward's staged rows,
// a_in), 1 BN(act) of a piecewise-linear act, 2 + dropout, 3 any activation
static int dw_prologue(const rt_linear_bwd_args& a) {
    if (a.prev_mode == 0 || a.a_in) return 0;
    return !act_is_piecewise_linear(a.prev_act) ? 3 : (a.prev_drop_p > 0.f ? 2 : 1);
}
// two sets whose prologues cannot share a kernel (a raw input and a
// transformed one: prologue 3 ⊇ 2 ⊇ 1, but 0 is disjoint): they run as two
// single-set launches, each with its own row-split plan
// (rt_linear_bwd_dw_splits follows the same rule)
static bool dw_mixed(const rt_linear_bwd_args* args, int n_args) {
    return n_args == 2 && (dw_prologue(args[0]) == 0) != (dw_prologue(args[1]) == 0);
}

// one dW launch over n_args sets that share a prologue family; dzf: the dz
// fusion decided for the whole call (the dz launch decided it jointly too)
static int dw_launch(const rt_linear_bwd_args* args, int n_args, bool dzf, hipStream_t st) {
    mlp::BwdLaunch L{};
    unsigned blocks[2] = {0u, 0u};
    int pro = -1;
    bool small_k = true;
    for (int g = 0; g < n_args; ++g) small_k = small_k && args[g].k <= 32;
    unsigned tns[2] = {1u, 1u}, tks[2] = {1u, 1u};
    int64_t nsplit[2] = {0, 0}, rps = mlp::DW_R;
    dw_plan(args, n_args, small_k, tns, tks, nsplit, rps);
    for (int g = 0; g < n_args; ++g) {
        const rt_linear_bwd_args& a = args[g];
        const int64_t nb = static_cast<int64_t>(tns[g]) * tks[g] * nsplit[g];
        if (nb > (1ll << 30)) return RT_ERR_UNSUPPORTED;
        blocks[g] = static_cast<unsigned>(nb);
        (g ? L.tn1 : L.tn0) = tns[g] ? tns[g] : 1u;
        (g ? L.tk1 : L.tk0) = tks[g] ? tks[g] : 1u;
        (g ? L.rps1 : L.rps0) = rps;
        // one kernel for both: prologue 3 ⊇ 2 ⊇ 1 (dropout p = 0 keeps everything)
        const int p = dw_prologue(a);
        pro = p > pro ? p : pro;
        const float* asrc = a.a_in ? a.a_in : a.src;
        const int ald = a.a_in ? a.k : a.ld_src;
        (g ? L.vec1 : L.vec0) = (a.n % 4) == 0 && (a.k % 4) == 0 && (ald % 4) == 0 &&
                                (reinterpret_cast<uintptr_t>(asrc) & 15) == 0 &&
                                (reinterpret_cast<uintptr_t>(a.dz_ws) & 15) == 0;
    }
    L.a0 = args[0];
    L.a1 = n_args > 1 ? args[1] : args[0];
    L.ngroups = n_args;
    if (n_args == 1) { L.tn1 = L.tn0; L.tk1 = L.tk0; L.rps1 = L.rps0; L.vec1 = L.vec0; }
    L.split = blocks[0];
    const unsigned total = blocks[0] + (n_args > 1 ? blocks[1] : 0u);
    if (total == 0) return RT_OK;
    const dim3 grid(total);
    const bool vec = L.vec0 && L.vec1;
#define RT_DW(BN, BK, P)                                                                                                 \
    do {                                                                                                                 \
        if (dzf) {                                                                                                       \
            if (vec) hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<BN, BK, P, true, true>), grid, dim3(mlp::DW_NT), 0, st, L);  \
            else hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<BN, BK, P, false, true>), grid, dim3(mlp::DW_NT), 0, st, L);     \
        } else {                                                                                                         \
            if (vec) hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<BN, BK, P, true, false>), grid, dim3(mlp::DW_NT), 0, st, L); \
            else hipLaunchKernelGGL((mlp::linear_bwd_dw_kernel<BN, BK, P, false, false>), grid, dim3(mlp::DW_NT), 0, st, L);    \
        }                                                                                                                \
    } while (0)
    if (small_k) {
        switch (pro) { case 0: RT_DW(128, 32, 0); break; case 1: RT_DW(128, 32, 1); break;
                       case 2: RT_DW(128, 32, 2); break; default: RT_DW(128, 32, 3); }
    } else {
        switch (pro) { case 0: RT_DW(64, 64, 0); break; case 1: RT_DW(64, 64, 1); break;
                       case 2: RT_DW(64, 64, 2); break; default: RT_DW(64, 64, 3); }
    }
#undef RT_DW
    return check_launch("linear_bwd_dw_kernel");
}

extern "C" int rt_linear_bwd_dw_f32_multi(const rt_linear_bwd_args* args, int n_args, void* stream) {
    if (!args || n_args < 1 || n_args > 2) return RT_ERR_INVALID;
#ifdef RT_NO_AIN
    rt_linear_bwd_args noa[2];
    for (int g = 0; g < n_args; ++g) { noa[g] = args[g]; noa[g].a_in = nullptr; }
    args = noa;
#endif
    for (int g = 0; g < n_args; ++g) {
        const int v = validate_bwd(&args[g]);
        if (v) return v;
        if (args[g].ids && args[g].prev_mode != 0) return RT_ERR_UNSUPPORTED;  // a gather feeds the first Linear only
    }
    hipStream_t st = as_stream(stream);
    // dz fusion as rt_linear_bwd_dz_f32_multi decided it for the same call: all sets or none
    const bool dzf = all_dz_fusable(args, n_args);
    if (dw_mixed(args, n_args)) {
        const int r0 = dw_launch(&args[0], 1, dzf, st);
        return r0 ? r0 : dw_launch(&args[1], 1, dzf, st);
    }
    return dw_launch(args, n_args, dzf, st);
}

extern "C" int rt_linear_bwd_dw_splits(const rt_linear_bwd_args* args, int n_args, int64_t* splits) {
    if (!args || !splits || n_args < 1 || n_args > 2) return RT_ERR_INVALID;
#ifdef RT_NO_DW_PART  // A/B build: callers keep the atomic dW adds
    return RT_ERR_UNSUPPORTED;
#endif
    bool small_k = true;
    for (int g = 0; g < n_args; ++g) {
        const int v = validate_bwd(&args[g]);
        if (v) return v;
        small_k = small_k && args[g].k <= 32;
    }
    unsigned tns[2] = {1u, 1u}, tks[2] = {1u, 1u};
    int64_t nsplit[2] = {0, 0}, rps = mlp::DW_R;
    if (dw_mixed(args, n_args)) {  // two single-set launches, two plans
        for (int g = 0; g < 2; ++g) {
            dw_plan(&args[g], 1, args[g].k <= 32, tns, tks, nsplit, rps);
            splits[g] = nsplit[0];
        }
        return RT_OK;
    }
    dw_plan(args, n_args, small_k, tns, tks, nsplit, rps);
    for (int g = 0; g < n_args; ++g) splits[g] = nsplit[g];
    return RT_OK;
}

extern "C" int rt_linear_bwd_dw_f32(const rt_linear_bwd_args* args, void* stream) {
    return rt_linear_bwd_dw_f32_multi(args, 1, stream);
}

#ifdef RT_PHASE_PROBE
// diagnostic builds only (not part of the ABI header)
extern "C" int rt_probe_setup(void* buf, unsigned cap) {
    unsigned long long* p = static_cast<unsigned long long*>(buf);
    const unsigned zero[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mlp::g_probe_buf), &p, sizeof(p)) != hipSuccess) return RT_ERR_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(mlp::g_probe_cap), &cap, sizeof(cap)) != hipSuccess) return RT_ERR_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(mlp::g_probe_ctr), zero, sizeof(zero)) != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
}
extern "C" int rt_probe_count(unsigned* out) {  // 64 shard counters
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mlp::g_probe_ctr), 64 * sizeof(unsigned)) == hipSuccess ? RT_OK
                                                                                                       : RT_ERR_HIP;
}
#endif

extern "C" int rt_linear_bwd_f32(const rt_linear_bwd_args* args, void* stream) {
    const int rc = rt_linear_bwd_dz_f32(args, stream);
    return rc ? rc : rt_linear_bwd_dw_f32(args, stream);
}
