// Flat-IP top-K, candidate-buffer variant with LDS-sorted compaction (one
// query set of 32 per wave, 64-item LDS tiles, register prefetch). Included by
// topk_impl.h: the 16-bit scans and k > 32 use this kernel (the scan stays at
// ~130 VGPRs, so two waves per SIMD hide the LDS/VMEM latency).
// Same contract as flatip_topk_kernel in topk_impl.h.
#pragma once

namespace rt {
namespace topk {
namespace v1 {

constexpr int kQT = 128;   // queries per block
constexpr int kNT = 64;    // items per LDS tile

inline int cap_for(int k) {
    int c = 128;
    while (c < k + kNT) c <<= 1;
    return c;
}

// per-wave LDS scratch for compaction: kMaxCap candidates
template <typename T, int S>
struct Smem {
    static constexpr int DP = S * Mfma<T>::kK;
    static constexpr int LS = DP + 16 / static_cast<int>(sizeof(T));  // +16 B pad per row
    T tile[kNT * LS];
    Cand sortbuf[kWaves][kMaxCap];
    int cnt[kQT];
    float theta[kQT];
};

// compact query buffer `buf` (n entries, n <= cap) down to its top-k
__device__ inline void wave_compact(Cand* __restrict__ buf, int n, int k, Cand* sb, int& cnt_out,
                                    float& theta_out) {
    const int lane = threadIdx.x & 63;
    const int np = next_pow2(n > 64 ? n : 64);
    for (int e = lane; e < np; e += 64) sb[e] = e < n ? buf[e] : Cand{-INFINITY, kEmptyId};
    wave_lds_sync();
    wave_sort_lds(sb, np);
    const int keep = n < k ? n : k;
    for (int e = lane; e < keep; e += 64) buf[e] = sb[e];
    cnt_out = keep;
    theta_out = keep == k ? sb[k - 1].s : -INFINITY;
    wave_lds_sync();
}

template <typename T, int S>
__global__ __launch_bounds__(256) void flatip_topk_v1_kernel(Args a, int cap, int64_t items_per_split) {
    using M = Mfma<T>;
    using SM = Smem<T, S>;
    constexpr int KK = M::kK;
    constexpr int DP = SM::DP;
    constexpr int LS = SM::LS;
    constexpr int VEC = 16 / static_cast<int>(sizeof(T));  // elements per 16-byte load
    constexpr int TILE_VECS = kNT * (DP / VEC);
    constexpr int LOADS = (TILE_VECS + 255) / 256;
    __shared__ SM sm;

    const T* __restrict__ Q = reinterpret_cast<const T*>(a.Q);
    const T* __restrict__ X = reinterpret_cast<const T*>(a.X);
    const int d = a.d, k = a.k;
    const int64_t nq = a.nq;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int col = lane & 31;          // query column inside the wave
    const int half = lane >> 5;         // k half inside an MFMA step
    const int ql = wave * 32 + col;     // block-local query
    const int64_t q = static_cast<int64_t>(blockIdx.x) * kQT + ql;
    const bool q_ok = q < nq;
    const int split = blockIdx.y;
    const int64_t i_begin = static_cast<int64_t>(split) * items_per_split;
    const int64_t i_end = (i_begin + items_per_split) < a.nx ? (i_begin + items_per_split) : a.nx;
    const int row_vecs = d / VEC;

    // ---- query fragments in registers: B[k][query] ----
    typename M::frag qf[S];
    {
        const T* qrow = Q + (q_ok ? q : 0) * d;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k0 = (KK == 2) ? (2 * s + half) : (16 * s + 8 * half);
            if (q_ok && k0 < d) qf[s] = frag_from<T>(qrow + k0);
            else qf[s] = typename M::frag{};
        }
    }
    Cand* my_cand = a.cand + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * kQT * cap;
    Cand* my_sb = sm.sortbuf[wave];
    if (tid < kQT) {
        sm.cnt[tid] = 0;
        sm.theta[tid] = (static_cast<int64_t>(blockIdx.x) * kQT + tid < nq) ? -INFINITY : INFINITY;
    }
    const uint32_t* my_excl = (a.excl && q_ok) ? a.excl + q * a.excl_words : nullptr;

    // register prefetch of one tile (rows t0 .. t0+63, zero padded)
    uint4 pre[LOADS];
    auto fetch = [&](int64_t t0) {
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            const int e = tid + l * 256;
            const int r = e / (DP / VEC);
            const int c = e % (DP / VEC);
            const int64_t item = t0 + r;
            pre[l] = make_uint4(0, 0, 0, 0);
            if (e < TILE_VECS && item < i_end && c < row_vecs)
                pre[l] = *reinterpret_cast<const uint4*>(X + item * d + c * VEC);
        }
    };
    fetch(i_begin);

    for (int64_t t0 = i_begin; t0 < i_end; t0 += kNT) {
        __syncthreads();  // previous tile consumed; cnt/theta published
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            const int e = tid + l * 256;
            if (e < TILE_VECS) {
                const int r = e / (DP / VEC);
                const int c = e % (DP / VEC);
                *reinterpret_cast<uint4*>(sm.tile + r * LS + c * VEC) = pre[l];
            }
        }
        __syncthreads();
        if (t0 + kNT < i_end) fetch(t0 + kNT);  // overlaps the MFMA work below
        const float th = sm.theta[ql];
#pragma unroll
        for (int rt = 0; rt < kNT / 32; ++rt) {
            f32x16 acc = {};
            const T* arow = sm.tile + (rt * 32 + col) * LS + ((KK == 2) ? half : 8 * half);
#pragma unroll
            for (int s = 0; s < S; ++s) acc = M::run(frag_from<T>(arow + s * KK), qf[s], acc);
            // acc[r] = score(item row (r&3)+8(r>>2)+4*half of the sub-tile, query col)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = acc[r];
                const int64_t item = t0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (v > th && item < i_end) {
                    const bool skip = my_excl && ((my_excl[item >> 5] >> (item & 31)) & 1u);
                    if (!skip) {
                        const int slot = atomicAdd(&sm.cnt[ql], 1);
                        my_cand[ql * cap + slot] = Cand{v, static_cast<uint32_t>(item)};
                    }
                }
            }
        }
        __threadfence_block();
        // ---- compaction of this wave's queries whose buffer nears capacity ----
        const bool need = (lane < 32) && (sm.cnt[ql] > cap - kNT);
        uint64_t mask = __ballot(need);
        while (mask) {
            const int c = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int qq = wave * 32 + c;
            int nc;
            float nt;
            wave_compact(my_cand + qq * cap, sm.cnt[qq], k, my_sb, nc, nt);
            __threadfence_block();
            if (lane == 0) { sm.cnt[qq] = nc; sm.theta[qq] = nt; }
            __threadfence_block();
        }
    }
    __syncthreads();
    // ---- final selection for this wave's 32 queries ----
    float* os = a.out_s + static_cast<int64_t>(split) * nq * k;
    int64_t* oi = a.out_i + static_cast<int64_t>(split) * nq * k;
    for (int c = 0; c < 32; ++c) {
        const int qq = wave * 32 + c;
        const int64_t gq = static_cast<int64_t>(blockIdx.x) * kQT + qq;
        if (gq >= nq) break;
        const int n = sm.cnt[qq];
        const int np = next_pow2((n > k ? n : k) > 64 ? (n > k ? n : k) : 64);
        for (int e = lane; e < np; e += 64) my_sb[e] = e < n ? my_cand[qq * cap + e] : Cand{-INFINITY, kEmptyId};
        wave_lds_sync();
        wave_sort_lds(my_sb, np);
        for (int e = lane; e < k; e += 64) {
            const Cand cv = my_sb[e];
            const bool ok = cv.i != kEmptyId;
            os[gq * k + e] = ok ? cv.s : -FLT_MAX;
            oi[gq * k + e] = ok ? static_cast<int64_t>(cv.i) + a.id_offset : -1;
        }
        wave_lds_sync();
    }
}

template <typename T, int S>
int launch_S(const Args& a, int cap, int splits, int64_t items_per_split, hipStream_t st) {
    dim3 grid(static_cast<unsigned>((a.nq + kQT - 1) / kQT), static_cast<unsigned>(splits));
    hipLaunchKernelGGL((flatip_topk_v1_kernel<T, S>), grid, dim3(256), 0, st, a, cap, items_per_split);
    return check_launch("flatip_topk_v1_kernel");
}

}  // namespace v1
}  // namespace topk
}  // namespace rt
