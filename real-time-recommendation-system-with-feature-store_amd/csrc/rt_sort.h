// Wave-level (64-lane) bitonic sorts of (score, id) candidates.
// Order: "better first" = score descending, then id ascending — the order in
// which Faiss IndexFlatIP reports results (lower id wins exact ties).
//
// wave_sort_lds: candidates in LDS (any power-of-two n); used by topk_merge.
// wave_sort_regs<E>: 64·E candidates held E per lane in registers (element
//   index = lane·E + j); strides < E are register compare-swaps, larger ones
//   one cross-lane shuffle per element — no LDS round trips, which is what the
//   top-K compaction/final selection spends its time on.
#pragma once

#include "rt_common.h"

namespace rt {

struct Cand {
    float s;
    uint32_t i;
};

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) { return better(a.s, a.i, b.s, b.i); }

// Sort buf[0, n) (n a power of two >= 2) in LDS, better first. Whole wave calls.
__device__ inline void wave_sort_lds(Cand* buf, int n) {
    const int lane = threadIdx.x & 63;
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int p = lane; p < (n >> 1); p += 64) {
                const int lo = ((p & ~(stride - 1)) << 1) | (p & (stride - 1));
                const int hi = lo + stride;
                const bool dir = (lo & size) == 0;
                const Cand a = buf[lo];
                const Cand b = buf[hi];
                if (better(b, a) == dir) {
                    buf[lo] = b;
                    buf[hi] = a;
                }
            }
            wave_lds_sync();
        }
    }
}

__device__ __forceinline__ int next_pow2(int x) {
    int p = 2;
    while (p < x) p <<= 1;
    return p;
}

// ---- register bitonic sort ------------------------------------------------
template <int E, int ST>
__device__ __forceinline__ void cas_in_regs(float (&s)[E], uint32_t (&id)[E], int lane, int size) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
        if ((j & ST) == 0) {
            const int jj = j | ST;
            const bool dir = (((lane * E) + j) & size) == 0;
            const bool hi_better = better(s[jj], id[jj], s[j], id[j]);
            if (hi_better == dir) {
                const float ts = s[j];
                const uint32_t ti = id[j];
                s[j] = s[jj];
                id[j] = id[jj];
                s[jj] = ts;
                id[jj] = ti;
            }
        }
    }
}

template <int E>
__device__ __forceinline__ void cas_in_dispatch(float (&s)[E], uint32_t (&id)[E], int lane, int size, int stride) {
    if constexpr (E >= 2) { if (stride == 1) { cas_in_regs<E, 1>(s, id, lane, size); return; } }
    if constexpr (E >= 4) { if (stride == 2) { cas_in_regs<E, 2>(s, id, lane, size); return; } }
    if constexpr (E >= 8) { if (stride == 4) { cas_in_regs<E, 4>(s, id, lane, size); return; } }
    if constexpr (E >= 16) { if (stride == 8) { cas_in_regs<E, 8>(s, id, lane, size); return; } }
}

template <int E>
__device__ __forceinline__ void cas_x_lanes(float (&s)[E], uint32_t (&id)[E], int lane, int size, int stride) {
    const int m = stride / E;  // partner lane = lane ^ m
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const float os = __shfl_xor(s[j], m, 64);
        const uint32_t oi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(id[j]), m, 64));
        const int idx = lane * E + j;
        const bool lower = (idx & stride) == 0;
        const bool dir = (idx & size) == 0;
        const bool mine_better = better(s[j], id[j], os, oi);
        const bool take = (lower == dir) ? !mine_better : mine_better;
        if (take) {
            s[j] = os;
            id[j] = oi;
        }
    }
}

// sort 64·E elements (element lane·E + j in s[j]/id[j] of that lane), better first
template <int E>
__device__ __forceinline__ void wave_sort_regs(float (&s)[E], uint32_t (&id)[E]) {
    const int lane = threadIdx.x & 63;
    constexpr int N = 64 * E;
    for (int size = 2; size <= N; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= E) cas_x_lanes<E>(s, id, lane, size, stride);
            else cas_in_dispatch<E>(s, id, lane, size, stride);
        }
    }
}

// ---- E = 2, every stage unrolled ---------------------------------------------
// The 128-entry sort of the v4 finish: lane distances 1 and 2 by DPP quad
// permutes (no LDS round trip), 4..16 by ds_swizzle in xor mode, 32 by
// ds_bpermute; each stage's per-lane direction is one compare of two lane bits.
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
    const int x = static_cast<int>(v);
    if constexpr (M == 1) return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
    else if constexpr (M == 2) return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
    else if constexpr (M < 32) return static_cast<uint32_t>(__builtin_amdgcn_ds_swizzle(x, 0x1F | (M << 10)));
    else return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(((threadIdx.x & 63) ^ 32) << 2, x));
}

// better() without short-circuit branches: three compares, mask logic, selects
__device__ __forceinline__ bool better_nb(float sa, uint32_t ia, float sb, uint32_t ib) {
    return (sa > sb) | ((sa == sb) & (ia < ib));
}

template <int SIZE, int STRIDE>
__device__ __forceinline__ void sort2_stage(float (&s)[2], uint32_t (&id)[2], int lane) {
    if constexpr (STRIDE == 1) {  // the lane's own pair (elements 2·lane, 2·lane + 1)
        const bool dir = ((2 * lane) & SIZE) == 0;
        const bool sw = better_nb(s[1], id[1], s[0], id[0]) == dir;
        const float s0 = s[0], s1 = s[1];
        const uint32_t i0 = id[0], i1 = id[1];
        s[0] = sw ? s1 : s0;
        s[1] = sw ? s0 : s1;
        id[0] = sw ? i1 : i0;
        id[1] = sw ? i0 : i1;
    } else {  // partner lane = lane ^ STRIDE / 2
        constexpr int M = STRIDE / 2;
        const bool keep_better = ((lane & M) == 0) == ((lane & (SIZE / 2)) == 0);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float os = __uint_as_float(xor_lane<M>(__float_as_uint(s[j])));
            const uint32_t oi = xor_lane<M>(id[j]);
            const bool take = keep_better != better_nb(s[j], id[j], os, oi);
            s[j] = take ? os : s[j];
            id[j] = take ? oi : id[j];
        }
    }
}

template <int SIZE, int STRIDE>
__device__ __forceinline__ void sort2_from(float (&s)[2], uint32_t (&id)[2], int lane) {
    sort2_stage<SIZE, STRIDE>(s, id, lane);
    if constexpr (STRIDE > 1) sort2_from<SIZE, STRIDE / 2>(s, id, lane);
    else if constexpr (SIZE < 128) sort2_from<SIZE * 2, SIZE>(s, id, lane);
}

// wave_sort_regs<2> with every stage unrolled
__device__ __forceinline__ void wave_sort_regs2(float (&s)[2], uint32_t (&id)[2]) {
    sort2_from<2, 1>(s, id, static_cast<int>(threadIdx.x & 63));
}

}  // namespace rt
