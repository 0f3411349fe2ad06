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

}  // namespace rt
