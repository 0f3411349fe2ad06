// On-device negative sampling (the GPU data feeder).
//
// Replaces sample_negative_items (src/data/movielens.py:488-512) as called per
// sample by MovieLensDataset.__getitem__ (src/training/datasets/movielens.py:
// 104-108): num_negatives items drawn uniformly WITHOUT replacement from the
// items the user has not interacted with; when that pool is smaller than
// num_negatives the whole pool is returned (here: in increasing id order, the
// remaining slots = -1).
//
// One wave per batch row, proposals counter-hashed from (seed, row, round, lane).
// Catalogues up to 65,536 items keep the user's positives and the accepted
// negatives in a per-wave LDS bitmap: all 64 lanes propose each round and the
// proposals whose bit they set first fill the open slots in lane order.
// Larger catalogues: lane j owns slot j, rejects a proposal that is one of the
// user's positives (binary search in the user's sorted CSR segment) or equals
// an accepted slot or a lower lane's same-round proposal, and retries.
// Distinctness is exact; the accepted set is uniform over the pool because each
// round's proposals are uniform and rejection only removes forbidden values.
#include "rt_common.h"

namespace rt {
namespace sampler {

constexpr int kMaxNeg = 64;
constexpr int kMaxRounds = 4096;

__device__ __forceinline__ uint32_t draw(uint64_t seed, int64_t row, int round, int j) {
    return static_cast<uint32_t>(mix64(seed ^ (static_cast<uint64_t>(row) * 0xD1B54A32D192ED03ull) ^
                                       (static_cast<uint64_t>(round) * 64u + static_cast<uint64_t>(j)) *
                                           0x9E3779B97F4A7C15ull) >> 32);
}

__device__ __forceinline__ bool contains(const int32_t* __restrict__ items, int64_t lo, int64_t hi, int32_t c) {
    int64_t a = lo, b = hi;
    while (a < b) {
        const int64_t mid = (a + b) >> 1;
        if (items[mid] < c) a = mid + 1;
        else b = mid;
    }
    return a < hi && items[a] == c;
}

// BITMAP: the catalogue fits a per-wave LDS bitmap (num_items <= kMaxBitmapItems):
// the user's positives are set in it once, accepted negatives are added as
// they are taken, so every membership test is one LDS read instead of a
// dependent binary search through global memory. The two forms do NOT produce
// the same negatives for the same seed: the bitmap form has all 64 lanes
// propose every round and fills the open slots in lane order (the surplus
// dropped), the search form has lane j own slot j. Both guarantee only the
// contract: distinct negatives, none a positive, uniform over the rest.
constexpr int64_t kMaxBitmapItems = 65536;

template <bool BITMAP>
__global__ __launch_bounds__(256) void sample_negatives_kernel(const int64_t* __restrict__ offsets,
                                                               const int32_t* __restrict__ items, int64_t n_users,
                                                               const int64_t* __restrict__ users, int64_t n,
                                                               int64_t num_items, int num_neg, uint64_t seed,
                                                               const uint64_t* __restrict__ seed_offset,
                                                               int64_t* __restrict__ out) {
    __shared__ int32_t acc_s[4][kMaxNeg];
    __shared__ int32_t prop_s[4][kMaxNeg];
    extern __shared__ uint32_t bits_s[];  // BITMAP: [4][words]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + w;
    if (row >= n) return;
    const uint64_t sd = seed + (seed_offset ? *seed_offset : 0ull);
    const int64_t u = users[row];
    int64_t lo = 0, hi = 0;
    if (u >= 0 && u < n_users) { lo = offsets[u]; hi = offsets[u + 1]; }
    const int64_t pool = num_items - (hi - lo);
    int64_t* o = out + row * num_neg;
    const int words = static_cast<int>((num_items + 31) / 32);
    uint32_t* const bits = bits_s + static_cast<int64_t>(w) * words;
    if constexpr (BITMAP) {
        for (int i = lane; i < words; i += 64) bits[i] = 0u;
        wave_lds_sync();
        // kPosUnroll independent loads per lane in flight before their LDS ors:
        // a heavy user's ~2,300 positives take 5 load round trips, not 37
        constexpr int kPosUnroll = 8;
        for (int64_t base = lo; base < hi; base += 64 * kPosUnroll) {
            int32_t v[kPosUnroll];
#pragma unroll
            for (int k = 0; k < kPosUnroll; ++k) {
                const int64_t i = base + k * 64 + lane;
                v[k] = i < hi ? items[i] : -1;
            }
#pragma unroll
            for (int k = 0; k < kPosUnroll; ++k)
                if (v[k] >= 0 && v[k] < num_items) atomicOr(&bits[v[k] >> 5], 1u << (v[k] & 31));
        }
        wave_lds_sync();
    }
    auto forbidden = [&](int32_t c) -> bool {
        if constexpr (BITMAP) return (bits[c >> 5] >> (c & 31)) & 1u;
        else return contains(items, lo, hi, c);
    };
    if (pool <= num_neg) {
        // the whole pool in id order (reference: `return negative_pool`), -1 padded
        int written = 0;
        for (int64_t base = 0; base < num_items && written < num_neg; base += 64) {
            const int64_t c = base + lane;
            const bool keep = c < num_items && !forbidden(static_cast<int32_t>(c));
            const uint64_t m = __ballot(keep);
            const int before = __popcll(m & ((1ull << lane) - 1ull));
            if (keep && written + before < num_neg) o[written + before] = c;
            written += __popcll(m);
        }
        for (int j = (written < num_neg ? written : num_neg) + lane; j < num_neg; j += 64) o[j] = -1;
        return;
    }
    if constexpr (BITMAP) {
        // Every lane proposes each round. A proposal is taken when its bit was
        // clear at its LDS or-with-return: positives and earlier-accepted
        // negatives are already set, and of equal proposals in one round only
        // the first to reach the LDS sees the bit clear. Taken proposals fill
        // the open slots in lane order; a round's surplus is dropped. Read in
        // (round, lane) order this is sequential uniform draws without
        // replacement from the pool, so the sample is uniform; a heavy user
        // (a third of the catalogue left) fills 16 slots in one round.
        int filled = 0;
        for (int round = 0; round < kMaxRounds && filled < num_neg; ++round) {
            const uint32_t r = draw(sd, row, round, lane);
            const int32_t c = static_cast<int32_t>((static_cast<uint64_t>(r) * static_cast<uint64_t>(num_items)) >> 32);
            const uint32_t bit = 1u << (c & 31);
            const bool ok = (atomicOr(&bits[c >> 5], bit) & bit) == 0u;
            const uint64_t m = __ballot(ok);
            const int slot = filled + __popcll(m & ((1ull << lane) - 1ull));
            if (ok && slot < num_neg) o[slot] = c;
            filled += __popcll(m);
        }
        for (int j = (filled < num_neg ? filled : num_neg) + lane; j < num_neg; j += 64) o[j] = -1;
        return;
    }
    int32_t mine = -1;
    const bool active = lane < num_neg;
    if (lane < kMaxNeg) acc_s[w][lane] = -1;
    for (int round = 0; round < kMaxRounds; ++round) {
        const bool want = active && mine < 0;
        if (!__ballot(want)) break;
        int32_t c = -1;
        if (want) {
            const uint32_t r = draw(sd, row, round, lane);
            c = static_cast<int32_t>((static_cast<uint64_t>(r) * static_cast<uint64_t>(num_items)) >> 32);
        }
        if (lane < kMaxNeg) prop_s[w][lane] = c;
        wave_lds_sync();
        bool ok = want && !forbidden(c);  // BITMAP: the accepted negatives are in the bitmap too
        if (ok) {
            for (int j = 0; j < (BITMAP ? lane : num_neg); ++j) {
                if ((!BITMAP && acc_s[w][j] == c) || (j < lane && prop_s[w][j] == c)) { ok = false; break; }
            }
        }
        wave_lds_sync();
        if (ok) {
            mine = c;
            if constexpr (BITMAP) atomicOr(&bits[c >> 5], 1u << (c & 31));
            else acc_s[w][lane] = c;
        }
        wave_lds_sync();
    }
    if (active) o[lane] = mine;  // -1 only if kMaxRounds ran out (pool > num_neg makes that vanishing)
}

// graph-captured epoch: the batch at the device cursor (rt_feeder_batch) and
// the post-step bookkeeping (rt_feeder_commit)
__global__ __launch_bounds__(256) void feeder_batch_kernel(const int64_t* __restrict__ order,
                                                           const int64_t* __restrict__ inter_u,
                                                           const int64_t* __restrict__ inter_m,
                                                           const int64_t* __restrict__ state, int64_t batch,
                                                           int64_t* __restrict__ users, int64_t* __restrict__ pos) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= batch) return;
    const int64_t row = order[state[0] * batch + t];
    users[t] = inter_u[row];
    pos[t] = inter_m[row];
}

__global__ void feeder_commit_kernel(const double* __restrict__ loss, double* __restrict__ losses, int64_t n_losses,
                                     int64_t* __restrict__ state) {
    if (threadIdx.x != 0) return;
    const int64_t b = state[0];
    if (b >= 0 && b < n_losses) losses[b] = loss[0];
    state[0] = b + 1;
    state[1] += 1;
}

}  // namespace sampler
}  // namespace rt

using namespace rt;

extern "C" int rt_sample_negatives(const int64_t* pos_offsets, const int32_t* pos_items, int64_t n_users,
                                   const int64_t* users, int64_t n, int64_t num_items, int num_neg, uint64_t seed,
                                   const uint64_t* seed_offset, int64_t* out, void* stream) {
    if (n < 0 || n_users < 0 || num_items <= 0 || num_items >= (1ll << 31) || num_neg <= 0) return RT_ERR_INVALID;
    if (num_neg > sampler::kMaxNeg) return RT_ERR_UNSUPPORTED;
    if (n == 0) return RT_OK;
    if (!pos_offsets || !users || !out || (!pos_items && n_users > 0)) return RT_ERR_INVALID;
    const dim3 grid(static_cast<unsigned>((n + 3) / 4));
    if (num_items <= sampler::kMaxBitmapItems) {
        const size_t lds = 4 * static_cast<size_t>((num_items + 31) / 32) * sizeof(uint32_t);
        hipLaunchKernelGGL(sampler::sample_negatives_kernel<true>, grid, dim3(256), lds, as_stream(stream),
                           pos_offsets, pos_items, n_users, users, n, num_items, num_neg, seed, seed_offset, out);
    } else {
        hipLaunchKernelGGL(sampler::sample_negatives_kernel<false>, grid, dim3(256), 0, as_stream(stream),
                           pos_offsets, pos_items, n_users, users, n, num_items, num_neg, seed, seed_offset, out);
    }
    return check_launch("sample_negatives_kernel");
}

extern "C" int rt_feeder_batch(const int64_t* order, const int64_t* inter_u, const int64_t* inter_m,
                               const int64_t* state, int64_t batch, int64_t* users, int64_t* pos, void* stream) {
    if (batch < 0 || (batch > 0 && (!order || !inter_u || !inter_m || !state || !users || !pos))) return RT_ERR_INVALID;
    if (batch == 0) return RT_OK;
    hipLaunchKernelGGL(sampler::feeder_batch_kernel, dim3(static_cast<unsigned>((batch + 255) / 256)), dim3(256), 0,
                       as_stream(stream), order, inter_u, inter_m, state, batch, users, pos);
    return check_launch("feeder_batch_kernel");
}

extern "C" int rt_feeder_commit(const double* loss, double* losses, int64_t n_losses, int64_t* state, void* stream) {
    if (!loss || !losses || !state || n_losses < 0) return RT_ERR_INVALID;
    hipLaunchKernelGGL(sampler::feeder_commit_kernel, dim3(1), dim3(64), 0, as_stream(stream), loss, losses, n_losses,
                       state);
    return check_launch("feeder_commit_kernel");
}
