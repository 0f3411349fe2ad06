// Row gather / scatter-add / Faiss-style L2 renorm (HBM-bound kernels).
//
// rt_gather_rows replaces the per-sample numpy fancy indexing of
// MovieLensDataset.__getitem__ (src/training/datasets/movielens.py:108-116) and
// the nn.Embedding lookup (src/models/two_tower.py:115-119, 257-261): rows are
// copied as 16-byte vectors, lanes flattened over (row, 16-B chunk) so a wave
// covers whole rows with contiguous 1 KiB accesses, one vector per thread over
// a grid that covers the whole gather (memory-level parallelism for the HBM
// roofline), nontemporal loads and stores.
#include "rt_common.h"

namespace rt {
namespace gather {

// one 16-B vector per thread and a grid covering every vector: the most
// independent row reads in flight chip-wide (probe, C5 shard shape: 5.1 TB/s
// at 4 per thread over 65,536 blocks -> 5.95 TB/s, tools/hip_probe/gather_probe.hip)
constexpr int kUnroll = 1;

// element vectors as clang ext_vector types (the nontemporal builtins need them)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// IDX: uint32_t when n_ids * vecs_per_row < 2^32 (cheap division), else int64_t
template <typename V, typename IDX>
__global__ __launch_bounds__(256) void gather_rows_kernel(const V* __restrict__ table, int64_t row_begin,
                                                          int64_t n_rows, uint32_t vecs_per_row,
                                                          const int64_t* __restrict__ ids, int64_t n_ids,
                                                          V* __restrict__ out, int32_t* __restrict__ oob) {
    const IDX total = static_cast<IDX>(n_ids) * vecs_per_row;
    const IDX stride = static_cast<IDX>(gridDim.x) * blockDim.x;
    IDX e0 = static_cast<IDX>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; e0 < total; e0 += stride * kUnroll) {
        V v[kUnroll];
        IDX dst[kUnroll];
        bool has[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const IDX e = e0 + u * stride;
            dst[u] = e;
            has[u] = e < total;
            if (has[u]) {
                const IDX r = e / vecs_per_row;
                const uint32_t c = static_cast<uint32_t>(e - r * vecs_per_row);
                const int64_t id = ids[r] - row_begin;
                if (id >= 0 && id < n_rows) {
                    v[u] = __builtin_nontemporal_load(table + id * vecs_per_row + c);  // read once
                } else {
                    v[u] = V{};
                    if (c == 0 && oob) atomicAdd(oob, 1);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
            if (has[u]) __builtin_nontemporal_store(v[u], out + dst[u]);  // streamed out, not re-read here
    }
}

__global__ __launch_bounds__(256) void scatter_add_rows_kernel(float* __restrict__ grad_table, int64_t n_rows,
                                                               int dim, const int64_t* __restrict__ ids,
                                                               int64_t n_ids, const float* __restrict__ g,
                                                               int64_t padding_idx) {
    const int64_t total = n_ids * dim;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += stride) {
        const int64_t r = e / dim;
        const int c = static_cast<int>(e - r * dim);
        const int64_t id = ids[r];
        if (id == padding_idx || id < 0 || id >= n_rows) continue;
        atomicAdd(grad_table + id * dim + c, g[e]);
    }
}

// faiss.normalize_L2 → fvec_renorm_L2, one lane per row, sequential fmaf chain
// (oracle/flatip.c orc_renorm_l2). Rows staged through LDS for coalescing.
__global__ __launch_bounds__(64) void l2_renorm_kernel(float* __restrict__ x, int64_t n, int d) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int ld = d + 1;  // odd stride: conflict-free per-lane row walk
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * 64;
    const int rows = static_cast<int>((n - r0) < 64 ? (n - r0) : 64);
    for (int e = threadIdx.x; e < rows * d; e += 64) {
        const int r = e / d, c = e - (e / d) * d;
        sm[r * ld + c] = x[(r0 + r) * d + c];
    }
    __syncthreads();
    if (threadIdx.x < rows) {
        float* row = sm + threadIdx.x * ld;
        float acc = 0.f;
        for (int j = 0; j < d; ++j) acc = __builtin_fmaf(row[j], row[j], acc);
        if (acc > 0.f) {
            // plain sqrtf / division: hipcc emits the correctly rounded sequences
            // (__fsqrt_rn lowers to the bare, not correctly rounded v_sqrt_f32)
            const float inv = 1.0f / sqrtf(acc);
            for (int j = 0; j < d; ++j) row[j] = row[j] * inv;
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < rows * d; e += 64) {
        const int r = e / d, c = e - (e / d) * d;
        x[(r0 + r) * d + c] = sm[r * ld + c];
    }
}

inline unsigned grid_for(int64_t work, int block, int64_t cap = 4096) {
    int64_t g = (work + block - 1) / block;
    if (g > cap) g = cap;  // grid-stride the rest
    if (g < 1) g = 1;
    return static_cast<unsigned>(g);
}

}  // namespace gather
}  // namespace rt

using namespace rt;

template <typename V>
static void launch_gather(const void* table, int64_t row_begin, int64_t n_rows, uint32_t vpr, const int64_t* ids,
                          int64_t n_ids, void* out, int32_t* oob, hipStream_t st) {
    // a grid over every vector keeps the most independent row reads in flight
    const unsigned grid = gather::grid_for(n_ids * vpr / gather::kUnroll, 256, 0x7FFFFFFF);
    if (n_ids * static_cast<int64_t>(vpr) + static_cast<int64_t>(grid) * 256 * gather::kUnroll < (1ll << 32)) {
        hipLaunchKernelGGL((gather::gather_rows_kernel<V, uint32_t>), dim3(grid), dim3(256), 0, st,
                           reinterpret_cast<const V*>(table), row_begin, n_rows, vpr, ids, n_ids,
                           reinterpret_cast<V*>(out), oob);
    } else {
        hipLaunchKernelGGL((gather::gather_rows_kernel<V, int64_t>), dim3(grid), dim3(256), 0, st,
                           reinterpret_cast<const V*>(table), row_begin, n_rows, vpr, ids, n_ids,
                           reinterpret_cast<V*>(out), oob);
    }
}

extern "C" int rt_gather_rows(const void* table, int64_t row_begin, int64_t n_rows, int64_t row_bytes,
                              const int64_t* ids, int64_t n_ids, void* out, int32_t* oob_count,
                              void* stream) {
    if (n_ids < 0 || n_rows < 0 || row_bytes <= 0 || (row_bytes & 3)) return RT_ERR_INVALID;
    if (n_ids == 0) return RT_OK;
    if (!ids || !out || (n_rows > 0 && !table)) return RT_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    const uintptr_t al = reinterpret_cast<uintptr_t>(table) | reinterpret_cast<uintptr_t>(out);
    if ((row_bytes & 15) == 0 && (al & 15) == 0) {
        launch_gather<gather::u32x4>(table, row_begin, n_rows, static_cast<uint32_t>(row_bytes / 16), ids, n_ids, out,
                             oob_count, st);
    } else if ((row_bytes & 7) == 0 && (al & 7) == 0) {
        launch_gather<gather::u32x2>(table, row_begin, n_rows, static_cast<uint32_t>(row_bytes / 8), ids, n_ids, out,
                             oob_count, st);
    } else {
        if (al & 3) return RT_ERR_INVALID;
        launch_gather<uint32_t>(table, row_begin, n_rows, static_cast<uint32_t>(row_bytes / 4), ids, n_ids, out,
                                oob_count, st);
    }
    return check_launch("gather_rows_kernel");
}

extern "C" int rt_scatter_add_rows_f32(float* grad_table, int64_t n_rows, int dim, const int64_t* ids,
                                       int64_t n_ids, const float* grad_out, int64_t padding_idx,
                                       void* stream) {
    if (n_ids < 0 || dim <= 0 || n_rows < 0) return RT_ERR_INVALID;
    if (n_ids == 0) return RT_OK;
    if (!grad_table || !ids || !grad_out) return RT_ERR_INVALID;
    hipLaunchKernelGGL(gather::scatter_add_rows_kernel, gather::grid_for(n_ids * dim, 256), dim3(256), 0,
                       as_stream(stream), grad_table, n_rows, dim, ids, n_ids, grad_out, padding_idx);
    return check_launch("scatter_add_rows_kernel");
}

extern "C" int rt_l2_renorm_f32(float* x, int64_t n, int d, void* stream) {
    if (n < 0 || d <= 0 || d > 512) return d > 512 ? RT_ERR_UNSUPPORTED : RT_ERR_INVALID;
    if (n == 0) return RT_OK;
    if (!x) return RT_ERR_INVALID;
    const unsigned blocks = static_cast<unsigned>((n + 63) / 64);
    const size_t lds = static_cast<size_t>(64) * (d + 1) * sizeof(float);
    hipLaunchKernelGGL(gather::l2_renorm_kernel, dim3(blocks), dim3(64), lds, as_stream(stream), x, n, d);
    return check_launch("l2_renorm_kernel");
}
