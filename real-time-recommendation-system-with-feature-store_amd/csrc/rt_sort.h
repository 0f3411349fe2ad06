// Wave-level (64-lane) bitonic sort of (score, id) candidates held in LDS.
// Order: "better first" = score descending, then id ascending — the order in
// which Faiss IndexFlatIP reports results (lower id wins exact ties).
// Rolled loops on purpose: the sort runs only when a candidate buffer fills,
// so code size / compile time matter more than its speed.
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

}  // namespace rt
