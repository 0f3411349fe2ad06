// In-batch-negative cross-entropy on 16-bit embeddings (config C5: bf16, D=256)
// with the scores on the 16-bit MFMA (v_mfma_f32_32x32x16_{bf16,f16}).
//
// Replaces, for 16-bit U/P and no explicit negatives,
//   in_batch_negative_loss (src/models/two_tower.py:453-479):
//     S = U·Pᵀ/τ ; L = mean_i CE(S_i, label off+i)
//   and its autograd backward  dU = dS·P/τ, dP = dSᵀ·U/τ, dS = (softmax(S) − I)/b.
// 16-bit × 16-bit products are exact in fp32 and the MFMA accumulates in fp32,
// so S equals the widened fp32 product up to summation order. dS is fp32; it
// enters the gradient MFMAs as a 16-bit hi + lo pair (bf16: to 2^-17 relative;
// f16 after a 2^15 scale that keeps small probabilities out of underflow), so
// the gradients keep close to fp32 accuracy.
//
// Three launches, flash-attention style (S is never stored):
//   lse  : fixed 32 users per wave (B operand in registers), items streamed
//          through LDS; online base-2 log-sum-exp per user and item split.
//   row  : same geometry; S recomputed, dS formed in registers and used, with
//          no lane movement, as the B operand of dUᵀ += Pᵀ·dS (the accumulator
//          layout of S IS the k-permuted operand layout); Pᵀ fragments come
//          from the same LDS image by ds_read_b64_tr_b16 (transposed reads).
//   col  : the mirror: fixed 32 items per wave, users streamed; dPᵀ += Uᵀ·dS.
// Item/user tiles arrive by LDS-DMA into a [NT][128-col] image per 128-column
// half whose 16-byte chunks are XOR-swizzled so that both the row reads
// (ds_read_b128) and the transposed reads are bank-conflict free.
// Every sub-tile issues all of its LDS fragment reads before the MFMAs that
// consume them (at one wave per SIMD a read an MFMA waits on exposes its whole
// latency); full stages are software-pipelined by one sub-tile (the S MFMAs of
// sub-tile t+1 overlap the exp/split VALU work of sub-tile t) and carry no tail
// masks or early exits.
// Gradient partials of each split are summed by a fixed-order reduce launch
// (deterministic, no atomics).
#include <float.h>

#include <type_traits>

#include "rt_common.h"

namespace rt {
namespace ib16 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;

template <typename T> struct M16;
template <> struct M16<__hip_bfloat16> {
    __device__ static f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(__attribute__((ext_vector_type(8))) __bf16, a),
                                                       __builtin_bit_cast(__attribute__((ext_vector_type(8))) __bf16, b),
                                                       c, 0, 0, 0);
    }
};
template <> struct M16<__half> {
    __device__ static f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(__attribute__((ext_vector_type(8))) _Float16, a),
                                                      __builtin_bit_cast(__attribute__((ext_vector_type(8))) _Float16, b),
                                                      c, 0, 0, 0);
    }
};

// accumulator element r of lane half h holds tile row krow(r) + 4h
__host__ __device__ constexpr int krow(int r) { return (r & 3) + 8 * (r >> 2); }

// ---- LDS image: per 128-column half, [NT rows][16 chunks of 16 B], chunk
// index XOR-swizzled by row (conflict-free row reads AND tr_b16 reads)
__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
template <int NT>
__device__ __forceinline__ int img_off(int half, int row, int ch) {
    return half * (NT * 256) + row * 256 + ((ch ^ swz(row)) << 4);
}

static __device__ const uint4 kZero16 = {0u, 0u, 0u, 0u};

template <typename P>
__device__ __forceinline__ uint32_t lds_addr(P* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)(p)));
}
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}
// same, wave-uniform base + 32-bit per-lane byte offset (SADDR form: no per-lane 64-bit address math)
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds_dst)
                 : "memory");
}
// transposed LDS read (ds_read_b64_tr_b16): for the 16-lane group of this lane,
// lane 4q+p addresses row q / columns 4p..4p+3 of a 4 x 16 block; lane i gets column i
__device__ __forceinline__ s16x4 tr_read(const char* lds, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds + byte_off));
}

// x → (hi, lo) 16-bit pair with x ≈ hi + lo; two elements packed per dword (lo
// element first); one v_cvt_pk per pair and rounding, RNE
template <typename T> struct Split;
template <> struct Split<__hip_bfloat16> {
    static constexpr float kScale = 1.f;  // bf16 keeps the fp32 exponent range
    static constexpr float kLog2Scale = 0.f;
    static constexpr float kLog2ScaleF = 0.f;  // ROWF: softmax weights up to 2^kSlack
    __device__ static void run(float x0, float x1, uint32_t& hp, uint32_t& lp) {
        typedef __bf16 b2 __attribute__((ext_vector_type(2)));
        const uint32_t hv = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{x0, x1}, b2));
        const float r0 = x0 - __builtin_bit_cast(float, hv << 16);
        const float r1 = x1 - __builtin_bit_cast(float, hv & 0xffff0000u);
        hp = hv;
        lp = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{r0, r1}, b2));
    }
};
template <> struct Split<__half> {
    static constexpr float kScale = 32768.f;  // dS·2^15 keeps small probabilities out of f16 underflow
    static constexpr float kLog2Scale = 15.f;
    // ROWF: weights up to 2^kSlack (lazy reference max), so 2^7 keeps them below
    // the f16 maximum; weights under 2^-31 of the reference underflow
    static constexpr float kLog2ScaleF = 7.f;
    __device__ static void run(float x0, float x1, uint32_t& hp, uint32_t& lp) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 hv = __builtin_convertvector(f32x2{x0, x1}, h2);
        const float r0 = x0 - static_cast<float>(hv[0]);
        const float r1 = x1 - static_cast<float>(hv[1]);
        hp = __builtin_bit_cast(uint32_t, hv);
        lp = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{r0, r1}, h2));
    }
};

// LSE: loss only; ROWF: the row log-sum-exp and dU in one pass (online
// softmax); COL: dP, against the finished lse2 (value 1 was the round-4 ROW
// pass, which took lse2 from a preceding LSE pass)
enum Pass { LSE = 0, COL = 2, ROWF = 3 };
// ROWF: the exponent reference is
// raised only when a sub-tile's max exceeds it by more than kSlack (base 2)
constexpr float kSlack = 8.f;

struct Args {
    const void* fixed;    // rows held as B operand (users for LSE/ROWF, items for COL)
    const void* stream;   // rows streamed through LDS
    int64_t n_fixed, n_stream;
    int d;
    int64_t off;          // label of user i is item off + i
    float c2;             // inv_tau * log2(e): base-2 logits
    float inv_tau;
    float w;              // d L / d CE_i = 1 / b
    int splits;
    int64_t per_split;    // streamed rows per split (multiple of NT)
    float2* part;         // LSE: [splits][n_fixed] (max2, sum) base 2
    float* diag2;         // LSE / ROWF: [n_fixed] x_ii (base-2 logit of the label)
    const float* lse2;    // COL: [b] base-2 log-sum-exp per user
    float* gpart;         // COL/ROWF: [splits][n_fixed][DP] gradient partials
                          // (ROWF: weighted by 2^(x - m_split), m_split in part[].x)
};

template <int DP, int PASS> struct Geo {
    static constexpr int S16 = DP / 16;                 // 16-wide k-steps of a dot
    // gradient passes at DP=256 hold 8 accumulator tiles (128 registers): one
    // wave per SIMD with the 512-register file; everything else two per SIMD
    static constexpr int WAVES = (PASS != 0 && DP > 128) ? 4 : 8;
    // streamed rows per LDS stage: 128 for the one-wave-per-SIMD gradient passes
    // (4 sub-tiles to pipeline over), 64 where two waves per SIMD share the registers
    static constexpr int NT = (DP > 128) ? 128 : 64;
    static constexpr int SUB = NT / 32;                 // 32-row sub-tiles per stage
    static constexpr int DB = DP / 32;                  // 32-wide d blocks of the gradient
    static constexpr int FT = 32 * WAVES;               // fixed rows per block
    static constexpr int TILE_BYTES = NT * DP * 2;
    static constexpr int DMA_PER_WAVE = TILE_BYTES / 1024 / WAVES;
    static_assert(DMA_PER_WAVE * 1024 * WAVES == TILE_BYTES, "tile must split into whole DMA pieces");
};

template <typename T, int DP, int PASS>
__global__ __launch_bounds__((Geo<DP, PASS>::WAVES * 64)) void ib16_kernel(Args a) {
    using G = Geo<DP, PASS>;
    using MM = M16<T>;
    constexpr int S16 = G::S16, NT = G::NT, DPW = G::DMA_PER_WAVE;
    __shared__ __attribute__((aligned(1024))) char tile[2][G::TILE_BYTES];
    __shared__ __attribute__((aligned(16))) float tlse[2][NT];  // COL: lse2 of the streamed users

    const T* __restrict__ F = reinterpret_cast<const T*>(a.fixed);
    const T* __restrict__ X = reinterpret_cast<const T*>(a.stream);
    const int d = a.d;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 31, h = lane >> 5;
    const int split = static_cast<int>(blockIdx.x % static_cast<unsigned>(a.splits));
    const int64_t fblk = blockIdx.x / static_cast<unsigned>(a.splits);
    const int64_t f = fblk * G::FT + wave * 32 + col;  // this lane's fixed row (its MFMA column)
    const bool fok = f < a.n_fixed;
    const int64_t i_begin = static_cast<int64_t>(split) * a.per_split;
    const int64_t i_end = (i_begin + a.per_split) < a.n_stream ? (i_begin + a.per_split) : a.n_stream;
    const int row_vecs = d / 8;

    // fixed-row fragments: B[k = 16s + 8h + j][col]
    s16x8 qf[S16];
    {
        const T* fr = F + (fok ? f : 0) * d;
#pragma unroll
        for (int s = 0; s < S16; ++s) {
            const int k0 = 16 * s + 8 * h;
            if (fok && k0 < d) qf[s] = __builtin_bit_cast(s16x8, *reinterpret_cast<const uint4*>(fr + k0));
            else qf[s] = s16x8{};
        }
    }

    // per-pass state
    float run_m = -INFINITY, run_s = 0.f, dg = 0.f;  // LSE (base 2), diag
    f32x16 gacc[G::DB];                               // ROWF/COL: gradient tile per 32-col d block
    if constexpr (PASS != LSE) {
#pragma unroll
        for (int i = 0; i < G::DB; ++i) gacc[i] = f32x16{};
    }
    // a padding lane (fixed row past the end) only feeds its own, never
    // stored, gradient column, so it needs no mask
    // ROWF: run_m is the exponent reference (shared by the two lane halves of a
    // fixed row), run_s this half's sum of 2^(x - run_m)·2^kLog2ScaleF
    const int64_t lab_row = f + a.off;  // LSE / ROWF: the item that is this user's label
    // wave-uniform: the wave's 32 label items are [lab0, lab0 + 32)
    const int64_t lab0 = fblk * G::FT + static_cast<int64_t>(__builtin_amdgcn_readfirstlane(wave)) * 32 + a.off;

    // ---- LDS-DMA of one stage: 1 KiB per wave-instruction into the lane-linear image ----
    const uint32_t wave_u = __builtin_amdgcn_readfirstlane(wave);
    const bool full_rows = (d == DP);  // no zero-filled columns: fixed per-lane offsets
    // this lane's byte offset of DMA piece j from the stage's first row
    // (recomputed per stage: the gradient passes have no registers to keep 16)
    auto voff = [&](int j) {
        const int o = (wave * DPW + j) * 1024 + lane * 16;
        const int half = o / (NT * 256);
        const int oo = o - half * (NT * 256);
        const int r = oo >> 8;
        const int c = half * 16 + (((oo & 255) >> 4) ^ swz(r));
        return static_cast<uint32_t>(r * d * 2 + c * 16);
    };
    auto fetch = [&](int64_t t0, int buf) {
        const uint32_t base = lds_addr(&tile[buf][0]) + wave_u * (DPW * 1024);
        if (full_rows && t0 + NT <= a.n_stream) {
            const void* sb = X + t0 * d;
#pragma unroll
            for (int j = 0; j < DPW; ++j) glds16_s(sb, voff(j), base + j * 1024);
        } else {  // zero-filled columns past d and/or rows clamped at the split end
#pragma unroll
            for (int j = 0; j < DPW; ++j) {
                const int o = (wave * DPW + j) * 1024 + lane * 16;
                const int half = o / (NT * 256);
                const int oo = o - half * (NT * 256);
                const int r = oo >> 8;
                const int c = half * 16 + (((oo & 255) >> 4) ^ swz(r));  // global 16-B chunk of the row
                int64_t item = t0 + r;
                item = item < i_end ? item : i_end - 1;
                const void* src = c < row_vecs ? static_cast<const void*>(X + item * d + c * 8)
                                               : static_cast<const void*>(&kZero16);
                glds16(src, base + j * 1024);
            }
        }
        if constexpr (PASS == COL) {  // NT lse2 values, 16 B per lane (the array is padded past b)
            if (wave == 0 && lane < NT / 4) glds16(a.lse2 + t0 + 4 * lane, lds_addr(&tlse[buf][0]));
        }
    };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // ---- pieces of one 32-row sub-tile rt of the stage image tl ----
    auto load_s = [&](const char* tl, int rt, s16x8 (&af)[S16]) {  // A fragments of the S tile
        const int row = rt * 32 + col;
#pragma unroll
        for (int s = 0; s < S16; ++s) {
            const int cg = 2 * s + h;
            af[s] = __builtin_bit_cast(s16x8, *reinterpret_cast<const uint4*>(tl + img_off<NT>(cg >> 4, row, cg & 15)));
        }
        __builtin_amdgcn_sched_barrier(0);  // keep every read issued ahead of the MFMAs
    };
    // S tile: acc[r] = <stream row sub0 + krow(r) + 4h, fixed row f>
    auto mma_s = [&](const s16x8 (&af)[S16]) {
        f32x16 acc = {};
#pragma unroll
        for (int s = 0; s < S16; ++s) acc = MM::run(af[s], qf[s], acc);
        return acc;
    };
    // transposed streamed-row fragments for the gradient: element j of half h = row
    // 16·s2 + 8(j>>2) + 4h + (j&3)
    auto load_g = [&](const char* tl, int rt, s16x8 (&ga)[G::DB][2]) {
        const int g16 = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
#pragma unroll
        for (int db = 0; db < G::DB; ++db) {
            const int half = db >> 2;
            const int c0 = ((db & 3) * 32 + 16 * (g16 & 1)) >> 3;  // chunk of the group's 16 columns
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int r0 = rt * 32 + 16 * s2 + 4 * h;
                const s16x4 lo4 = tr_read(tl, img_off<NT>(half, r0 + q, c0 + (p >> 1)) + 8 * (p & 1));
                const s16x4 hi4 = tr_read(tl, img_off<NT>(half, r0 + 8 + q, c0 + (p >> 1)) + 8 * (p & 1));
                ga[db][s2] = s16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            }
        }
    };
    // this lane's label row inside the sub-tile at sub0, relative to its lane half
    auto lab_pos = [&](int64_t sub0) {
        const int64_t dl = lab_row - sub0;
        return (dl >= 0 && dl < 32 ? static_cast<int>(dl) : 64) - 4 * h;
    };
    // LSE: online base-2 log-sum-exp over the sub-tile's valid rows (left of 32)
    auto lse_update = [&](const f32x16& acc, int64_t sub0, int left) {
        const int lim = left - 4 * h;  // row krow(r) + 4h is valid <=> krow(r) < lim
        float x[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) x[r] = acc[r] * a.c2;
        if (left < 32) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (krow(r) >= lim) x[r] = -INFINITY;
        }
        float mx = x[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, x[r]);
        const float mn = fmaxf(run_m, mx);
        // raw v_exp_f32: arguments are <= 0, results below 2^-126 flush to 0
        // (negligible next to the max term's 1)
        float s = (mn == -INFINITY) ? 0.f : run_s * __builtin_amdgcn_exp2f(run_m - mn);
#pragma unroll
        for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(x[r] - mn);
        run_m = mn;
        run_s = s;
        const int lr = lab_pos(sub0);
        if (fok && static_cast<unsigned>(lr) < 28u) {  // this lane holds its label's logit
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (krow(r) == lr) dg = x[r];
        }
    };
    // ROWF: the sub-tile's max per fixed row (both lane halves), the lazy
    // reference raise with its rescale of the accumulators (wave-uniform
    // branch, taken on a wave's first sub-tiles and rarely after), the label logit
    auto rowf_prep = [&](const f32x16& acc, int64_t sub0, int left) {
        const int lim = left - 4 * h;
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (left >= 32 || krow(r) < lim) mx = fmaxf(mx, acc[r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * a.c2;  // c2 > 0
        const bool up = mx > run_m + kSlack;
        if (__builtin_expect(__ballot(up) != 0ull, 0)) {
            asm volatile("; ib16 rowf rescale" ::: "memory");  // a real branch: never if-converted
            const float fct = up ? __builtin_amdgcn_exp2f(run_m - mx) : 1.f;  // 0 from -inf
            // the accumulators stay in AGPRs: each element is read, scaled and
            // written back through one VGPR (a VALU multiply on the vector
            // would make the allocator move all 128 of them into VGPRs)
#pragma unroll
            for (int db = 0; db < G::DB; ++db)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float v = gacc[db][r], t;
                    asm volatile("v_accvgpr_read_b32 %0, %1\n\tv_mul_f32 %0, %0, %2\n\tv_accvgpr_write_b32 %1, %0"
                                 : "=&v"(t), "+a"(v)
                                 : "v"(fct));
                    gacc[db][r] = v;
                }
            run_s *= fct;
            run_m = up ? mx : run_m;
        }
        if (lab0 + 32 > sub0 && lab0 < sub0 + 32) {  // wave-uniform
            const int lr = lab_pos(sub0);
            if (fok && static_cast<unsigned>(lr) < 28u) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (krow(r) == lr) dg = acc[r] * a.c2;
            }
        }
    };
    // ROWF/COL: the softmax part of dS, 2^(x − reference)·scale, in registers as
    // 16-bit hi + lo (the label term −[label] is applied by the reduce launch)
    auto make_ds = [&](const f32x16& acc, const float* tls, int rt, int64_t sub0, int left, s16x8 (&bh)[2],
                       s16x8 (&bl)[2]) {
        float lse_r[16];
        if constexpr (PASS == COL) {  // users are the streamed rows: lse2 per row, from LDS
            const float* t = tls + rt * 32;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 v = *reinterpret_cast<const float4*>(t + 8 * g + 4 * h);
                lse_r[4 * g] = v.x; lse_r[4 * g + 1] = v.y; lse_r[4 * g + 2] = v.z; lse_r[4 * g + 3] = v.w;
            }
        }
        float ds[16];
        if constexpr (PASS == ROWF) {  // 2^(x − run_m)·2^kLog2ScaleF, summed into run_s
            const float l = run_m - Split<T>::kLog2ScaleF;
#pragma unroll
            for (int r = 0; r < 16; ++r) ds[r] = __builtin_amdgcn_exp2f(acc[r] * a.c2 - l);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float l = lse_r[r] - Split<T>::kLog2Scale;
                ds[r] = __builtin_amdgcn_exp2f(acc[r] * a.c2 - l);
            }
        }
        if (left < 32) {
            const int lim = left - 4 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (krow(r) >= lim) ds[r] = 0.f;
        }
        if constexpr (PASS == ROWF) {
            float t = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) t += ds[r];
            run_s += t;
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            uint32_t hp[4], lp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) Split<T>::run(ds[8 * s2 + 2 * j], ds[8 * s2 + 2 * j + 1], hp[j], lp[j]);
            bh[s2] = __builtin_bit_cast(s16x8, make_uint4(hp[0], hp[1], hp[2], hp[3]));
            bl[s2] = __builtin_bit_cast(s16x8, make_uint4(lp[0], lp[1], lp[2], lp[3]));
        }
    };
    // gradient: gaccᵀ[d][f] += Σ_rows X[row][d] · dS[row][f]
    auto mma_g = [&](const s16x8 (&ga)[G::DB][2], const s16x8 (&bh)[2], const s16x8 (&bl)[2]) {
#pragma unroll
        for (int db = 0; db < G::DB; ++db)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                gacc[db] = MM::run(ga[db][s2], bh[s2], gacc[db]);
                gacc[db] = MM::run(ga[db][s2], bl[s2], gacc[db]);
            }
    };

    // LSE: a full stage, software-pipelined by one sub-tile: the S MFMAs of
    // sub-tile rt+1 are independent of sub-tile rt's exp VALU work and overlap it
    auto stage_full = [&](int64_t t0, const char* tl) {
        s16x8 af[S16];
        load_s(tl, 0, af);
        f32x16 acc = mma_s(af);
#pragma unroll
        for (int rt = 0; rt < G::SUB; ++rt) {
            const int64_t sub0 = t0 + rt * 32;
            f32x16 acc_n = {};
            if (rt + 1 < G::SUB) {
                load_s(tl, rt + 1, af);
                acc_n = mma_s(af);
            }
            lse_update(acc, sub0, 32);
            acc = acc_n;
        }
    };
    // gradient passes, reads one sub-tile ahead, in place, and an explicit
    // issue pattern: once an S MFMA of rt+1 is issued its fragment registers
    // take a read of rt+2, once a gradient MFMA of rt is issued its transposed
    // fragment takes a read of rt+1, and the dS VALU of rt is spread over the
    // S MFMAs (5 per gap) — no read is waited for by the MFMA right after it
    auto stage_full_g = [&](int64_t t0, const char* tl, const float* tls) {
        s16x8 af[S16];
        load_s(tl, 0, af);
        f32x16 acc = mma_s(af);
        s16x8 ga[G::DB][2];
        load_g(tl, 0, ga);
        if (G::SUB > 1) load_s(tl, 1, af);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < G::SUB; ++rt) {
            const int64_t sub0 = t0 + rt * 32;
            if constexpr (PASS == ROWF) {
                rowf_prep(acc, sub0, 32);
                __builtin_amdgcn_sched_barrier(0);
            }
            f32x16 acc_n = {};
            if (rt + 1 < G::SUB) {
#pragma unroll
                for (int ss = 0; ss < S16; ++ss) acc_n = MM::run(af[ss], qf[ss], acc_n);
            }
            if (rt + 2 < G::SUB) {
                const int row = (rt + 2) * 32 + col;
#pragma unroll
                for (int ss = 0; ss < S16; ++ss) {
                    const int cg = 2 * ss + h;
                    af[ss] = __builtin_bit_cast(s16x8, *reinterpret_cast<const uint4*>(
                                                           tl + img_off<NT>(cg >> 4, row, cg & 15)));
                }
            }
            s16x8 bh[2], bl[2];
            make_ds(acc, tls, rt, sub0, 32, bh, bl);
            mma_g(ga, bh, bl);
            if (rt + 1 < G::SUB) load_g(tl, rt + 1, ga);
#pragma unroll
            for (int i = 0; i < S16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // VALU
            }
#pragma unroll
            for (int i = 0; i < 4 * G::DB; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            acc = acc_n;
        }
    };
    // the split's last, partial stage: sub-tile by sub-tile with row masks
    auto stage_tail = [&](int64_t t0, const char* tl, const float* tls) {
#pragma unroll
        for (int rt = 0; rt < G::SUB; ++rt) {
            const int64_t sub0 = t0 + rt * 32;
            if (sub0 >= i_end) break;  // block-uniform
            const int left = static_cast<int>(i_end - sub0 < 32 ? i_end - sub0 : 32);
            s16x8 af[S16];
            load_s(tl, rt, af);
            const f32x16 acc = mma_s(af);
            if constexpr (PASS == LSE) {
                lse_update(acc, sub0, left);
            } else {
                s16x8 ga[G::DB][2];
                load_g(tl, rt, ga);
                if constexpr (PASS == ROWF) rowf_prep(acc, sub0, left);
                s16x8 bh[2], bl[2];
                make_ds(acc, tls, rt, sub0, left, bh, bl);
                mma_g(ga, bh, bl);
            }
        }
    };

    // full stages in the loop, the partial one after it: one path through the
    // loop body keeps the accumulators in one register assignment
    if (i_begin < i_end) fetch(i_begin, 0);
    raw_barrier();
    int cur = 0;
    const int64_t t_full = i_begin + (i_end - i_begin) / NT * NT;  // end of the full stages
    int64_t t0 = i_begin;
    for (; t0 < t_full; t0 += NT) {
        if (t0 + NT < i_end) fetch(t0 + NT, cur ^ 1);
        if constexpr (PASS != LSE) stage_full_g(t0, tile[cur], tlse[cur]);
        else stage_full(t0, tile[cur]);
        raw_barrier();
        cur ^= 1;
    }
    if (t0 < i_end) stage_tail(t0, tile[cur], tlse[cur]);

    if constexpr (PASS == LSE) {
        // merge the two lane halves (same fixed row), write the split's partial
        const float om = __shfl_xor(run_m, 32, 64), os = __shfl_xor(run_s, 32, 64);
        const float mn = fmaxf(run_m, om);
        float s = 0.f;
        if (mn != -INFINITY) s = run_s * exp2f(run_m - mn) + os * exp2f(om - mn);
        const float dgo = __shfl_xor(dg, 32, 64);
        if (fok && h == 0) {
            a.part[static_cast<int64_t>(split) * a.n_fixed + f] = make_float2(mn, s);
            const int64_t lab = f + a.off;
            if (lab >= i_begin && lab < i_end) {
                const int64_t rr = lab - (i_begin + ((lab - i_begin) & ~31ll));
                a.diag2[f] = ((rr >> 2) & 1) ? dgo : dg;
            }
        }
    } else {
        if constexpr (PASS == ROWF) {  // the split's (reference, Σ 2^(x − reference)) and label logit
            const float sc = exp2f(-Split<T>::kLog2ScaleF);
            const float s_all = (run_s + __shfl_xor(run_s, 32, 64)) * sc;
            const float dgo = __shfl_xor(dg, 32, 64);
            if (fok && h == 0) {
                a.part[static_cast<int64_t>(split) * a.n_fixed + f] = make_float2(run_m, s_all);
                const int64_t lab = f + a.off;
                if (lab >= i_begin && lab < i_end) {
                    const int64_t rr = lab - (i_begin + ((lab - i_begin) & ~31ll));
                    a.diag2[f] = ((rr >> 2) & 1) ? dgo : dg;
                }
            }
        }
        // gaccᵀ[db][r] = grad[d = 32db + krow(r) + 4h][fixed row f] → partial [split][f][DP]
        if (fok) {
            const float gs = a.inv_tau * a.w /
                             (PASS == ROWF ? exp2f(Split<T>::kLog2ScaleF) : Split<T>::kScale);
            float* gp = a.gpart + (static_cast<int64_t>(split) * a.n_fixed + f) * DP;
#pragma unroll
            for (int db = 0; db < G::DB; ++db)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<float4*>(gp + 32 * db + 8 * g + 4 * h) =
                        make_float4(gacc[db][4 * g] * gs, gacc[db][4 * g + 1] * gs, gacc[db][4 * g + 2] * gs,
                                    gacc[db][4 * g + 3] * gs);
        }
    }
}

// lse2_i = log2 Σ_splits sum·2^max ; L += w_loss · mean_i (lse2_i − x_ii)/log2e
__global__ __launch_bounds__(256) void ib16_finalize_kernel(const float2* __restrict__ part, int splits, int64_t b,
                                                            const float* __restrict__ diag2, float* __restrict__ lse2,
                                                            double* __restrict__ loss_out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    double ce = 0.0;
    if (i < b) {
        float m = -INFINITY;
        for (int s = 0; s < splits; ++s) m = fmaxf(m, part[static_cast<int64_t>(s) * b + i].x);
        float sum = 0.f;
        for (int s = 0; s < splits; ++s) {
            const float2 v = part[static_cast<int64_t>(s) * b + i];
            if (v.x != -INFINITY) sum += v.y * exp2f(v.x - m);
        }
        const float l2 = m + log2f(sum);
        lse2[i] = l2;
        ce = static_cast<double>((l2 - diag2[i]) / kLog2e);
    }
    ce = wave_sum(ce);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ce;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = (red[0] + red[1] + red[2] + red[3]) / static_cast<double>(b);
        atomicAdd(&loss_out[0], t);
        atomicAdd(&loss_out[2], t);
    }
}

// out[r][c] = Σ_s wt_s·part[s][r][c] (fixed order) − coef·lab[r + lab_off][c]
// (the label term of dS = softmax − I, when row r + lab_off of lab exists),
// c < d; wt_s = 1, or with ROWF partials (ml non-NULL) 2^(ml[s][r].x − lse2[r]),
// the split's exponent reference over the row's log-sum-exp
template <typename T>
__global__ __launch_bounds__(256) void ib16_reduce_kernel(const float* __restrict__ part, int splits, int64_t rows,
                                                          int dp, int d, const T* __restrict__ lab, int64_t lab_off,
                                                          int64_t lab_rows, float coef, float* __restrict__ out,
                                                          const float2* __restrict__ ml,
                                                          const float* __restrict__ lse2) {
    const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
    const int64_t total = rows * d;
    if (e >= total) return;
    const int64_t r = e / d;
    const int c = static_cast<int>(e - r * d);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float l2 = ml ? lse2[r] : 0.f;
    for (int s = 0; s < splits; ++s) {
        float4 v = *reinterpret_cast<const float4*>(part + (static_cast<int64_t>(s) * rows + r) * dp + c);
        if (ml) {
            const float m = ml[static_cast<int64_t>(s) * rows + r].x;
            const float wt = m == -INFINITY ? 0.f : exp2f(m - l2);
            v.x *= wt; v.y *= wt; v.z *= wt; v.w *= wt;
        }
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    const int64_t lr = r + lab_off;
    if (lr >= 0 && lr < lab_rows) {
        const T* l = lab + lr * d + c;
        acc.x -= coef * static_cast<float>(l[0]);
        acc.y -= coef * static_cast<float>(l[1]);
        acc.z -= coef * static_cast<float>(l[2]);
        acc.w -= coef * static_cast<float>(l[3]);
    }
    *reinterpret_cast<float4*>(out + e) = acc;
}

inline int splits_for(int64_t fixed_blocks, int64_t n_stream, int nt) {
    int64_t s = (256 + fixed_blocks - 1) / fixed_blocks;  // ~1 block per CU
    const int64_t mx = (n_stream + 4 * nt - 1) / (4 * nt);  // >= 4 stages per split
    if (s > mx) s = mx;
    if (s > 64) s = 64;
    return static_cast<int>(s < 1 ? 1 : s);
}

struct PassPlan {
    int64_t fixed_blocks;
    int splits;
    int64_t per;  // streamed rows per split (multiple of NT)
};

inline PassPlan pass_plan(int64_t n_fixed, int64_t n_stream, int ft, int nt) {
    PassPlan q{};
    q.fixed_blocks = (n_fixed + ft - 1) / ft;
    q.splits = splits_for(q.fixed_blocks, n_stream, nt);
    q.per = ((n_stream + q.splits - 1) / q.splits + nt - 1) / nt * nt;
    q.splits = static_cast<int>((n_stream + q.per - 1) / q.per);
    return q;
}

struct Plan {
    int dp;
    PassPlan lse, row, col;
    size_t part_off, diag_off, lse_off, gp_off, bytes;
};

template <int DP>
inline Plan make_plan_t(int64_t b, int64_t nx) {
    Plan p{};
    p.dp = DP;
    p.lse = pass_plan(b, nx, Geo<DP, LSE>::FT, Geo<DP, LSE>::NT);
    p.row = pass_plan(b, nx, Geo<DP, ROWF>::FT, Geo<DP, ROWF>::NT);
    p.col = pass_plan(nx, b, Geo<DP, COL>::FT, Geo<DP, COL>::NT);
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    size_t o = 0;
    const int part_splits = p.lse.splits > p.row.splits ? p.lse.splits : p.row.splits;  // LSE or ROWF partials
    p.part_off = o; o += al(static_cast<size_t>(part_splits) * b * sizeof(float2));
    p.diag_off = o; o += al(static_cast<size_t>(b) * sizeof(float));
    // the COL pass DMAs NT lse2 values per stage: padded past b by a whole stage
    p.lse_off = o; o += al(static_cast<size_t>((b + 255) / 256 * 256 + 256) * sizeof(float));
    p.gp_off = o;
    const size_t g_row = static_cast<size_t>(p.row.splits) * b * DP * sizeof(float);
    const size_t g_col = static_cast<size_t>(p.col.splits) * nx * DP * sizeof(float);
    o += al(g_row > g_col ? g_row : g_col);
    p.bytes = o;
    return p;
}

inline Plan make_plan(int64_t b, int64_t nx, int d) {
    return d <= 128 ? make_plan_t<128>(b, nx) : make_plan_t<256>(b, nx);
}

}  // namespace ib16

// workspace for the 16-bit in-batch path (rt_inbatch_loss_fwd_bwd, n_neg = 0)
size_t ib16_workspace_bytes(int64_t b, int64_t nx, int d) { return ib16::make_plan(b, nx, d).bytes; }

template <typename T, int DP>
static int ib16_run_t(const void* u, const void* p, int64_t b, int64_t nx, int d, int64_t off, float inv_tau,
                      double* loss_out, float* du, float* dp, char* ws, const ib16::Plan& pl, hipStream_t st) {
    using namespace ib16;
    Args a{};
    a.d = d;
    a.off = off;
    a.c2 = inv_tau * kLog2e;
    a.inv_tau = inv_tau;
    a.w = 1.f / static_cast<float>(b);
    a.part = reinterpret_cast<float2*>(ws + pl.part_off);
    a.diag2 = reinterpret_cast<float*>(ws + pl.diag_off);
    float* lse2 = reinterpret_cast<float*>(ws + pl.lse_off);
    a.lse2 = lse2;
    a.gpart = reinterpret_cast<float*>(ws + pl.gp_off);
    const dim3 blk_l(Geo<DP, LSE>::WAVES * 64), blk_r(Geo<DP, ROWF>::WAVES * 64), blk_c(Geo<DP, COL>::WAVES * 64);
    auto grid = [](const PassPlan& q) { return dim3(static_cast<unsigned>(q.fixed_blocks * q.splits)); };
    a.fixed = u; a.stream = p; a.n_fixed = b; a.n_stream = nx;
    int rc;
    const float coef = inv_tau * a.w;  // d L/d S_label = −w, times 1/τ
    if (!du) {  // loss only: the LSE pass
        a.splits = pl.lse.splits; a.per_split = pl.lse.per;
        hipLaunchKernelGGL((ib16_kernel<T, DP, LSE>), grid(pl.lse), blk_l, 0, st, a);
        if ((rc = check_launch("ib16_kernel<lse>"))) return rc;
        hipLaunchKernelGGL(ib16_finalize_kernel, dim3(static_cast<unsigned>((b + 255) / 256)), dim3(256), 0, st,
                           a.part, pl.lse.splits, b, a.diag2, lse2, loss_out);
        return check_launch("ib16_finalize_kernel");
    }
    // LSE and dU in one pass (online softmax per split), then the row
    // log-sum-exp, the loss and the split-weighted dU reduce
    a.splits = pl.row.splits; a.per_split = pl.row.per;
    hipLaunchKernelGGL((ib16_kernel<T, DP, ROWF>), grid(pl.row), blk_r, 0, st, a);
    if ((rc = check_launch("ib16_kernel<rowf>"))) return rc;
    hipLaunchKernelGGL(ib16_finalize_kernel, dim3(static_cast<unsigned>((b + 255) / 256)), dim3(256), 0, st, a.part,
                       pl.row.splits, b, a.diag2, lse2, loss_out);
    if ((rc = check_launch("ib16_finalize_kernel"))) return rc;
    hipLaunchKernelGGL(ib16_reduce_kernel<T>, dim3(static_cast<unsigned>((b * d / 4 + 255) / 256)), dim3(256), 0, st,
                       a.gpart, pl.row.splits, b, DP, d, reinterpret_cast<const T*>(p), off, nx, coef, du,
                       static_cast<const float2*>(a.part), static_cast<const float*>(lse2));
    if ((rc = check_launch("ib16_reduce_kernel(du)"))) return rc;
    // column pass: dP (items fixed, users streamed)
    a.fixed = p; a.stream = u; a.n_fixed = nx; a.n_stream = b;
    a.splits = pl.col.splits; a.per_split = pl.col.per;
    hipLaunchKernelGGL((ib16_kernel<T, DP, COL>), grid(pl.col), blk_c, 0, st, a);
    if ((rc = check_launch("ib16_kernel<col>"))) return rc;
    hipLaunchKernelGGL(ib16_reduce_kernel<T>, dim3(static_cast<unsigned>((nx * d / 4 + 255) / 256)), dim3(256), 0, st,
                       a.gpart, pl.col.splits, nx, DP, d, reinterpret_cast<const T*>(u), -off, b, coef, dp,
                       static_cast<const float2*>(nullptr), static_cast<const float*>(nullptr));
    return check_launch("ib16_reduce_kernel(dp)");
}

// 16-bit in-batch CE (n_neg = 0). d % 8 == 0, d <= 256; 16-B aligned rows.
int ib16_run(const void* u, const void* p, int dtype, int64_t b, int64_t nx, int d, int64_t off, float inv_tau,
             double* loss_out, float* du, float* dp, void* ws, size_t ws_bytes, hipStream_t st) {
    const ib16::Plan pl = ib16::make_plan(b, nx, d);
    if (!ws || ws_bytes < pl.bytes) return RT_ERR_WORKSPACE;
    char* w = reinterpret_cast<char*>(ws);
    if (dtype == RT_BF16) {
        return pl.dp == 128 ? ib16_run_t<__hip_bfloat16, 128>(u, p, b, nx, d, off, inv_tau, loss_out, du, dp, w, pl, st)
                            : ib16_run_t<__hip_bfloat16, 256>(u, p, b, nx, d, off, inv_tau, loss_out, du, dp, w, pl, st);
    }
    return pl.dp == 128 ? ib16_run_t<__half, 128>(u, p, b, nx, d, off, inv_tau, loss_out, du, dp, w, pl, st)
                        : ib16_run_t<__half, 256>(u, p, b, nx, d, off, inv_tau, loss_out, du, dp, w, pl, st);
}

}  // namespace rt
