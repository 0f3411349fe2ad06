// Shared device/host helpers for librtrec_hip.so (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "rtrec_hip.h"

#define RT_WAVE 64

namespace rt {

// thread-local record of the last failing HIP call (rt_last_error)
void set_last_error(const char* what, hipError_t e);

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(what, e);
        return RT_ERR_HIP;
    }
    return RT_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- element conversions (widen to f32 on load) ----
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__half x) { return __half2float(x); }
__device__ __forceinline__ float to_f32(__hip_bfloat16 x) { return __bfloat162float(x); }

__device__ __forceinline__ float bits_f16_to_f32(uint16_t b) {
    return __half2float(__ushort_as_half(b));
}
__device__ __forceinline__ float bits_bf16_to_f32(uint16_t b) {
    return __uint_as_float(static_cast<uint32_t>(b) << 16);
}

// ---- wave reductions (64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// order LDS traffic of one wave: DS ops of a wave complete in order; this also
// stops the compiler from hoisting reads above earlier writes by other lanes
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- counter-based RNG for dropout masks (splitmix64 finaliser) ----
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// keep element (row, col) of a dropout layer with probability 1-p
// (32-bit murmur3 finaliser over seed/row/col: ~10 VALU ops per element)
__device__ __forceinline__ bool dropout_keep(uint64_t seed, int64_t row, int col, float p) {
    uint32_t h = static_cast<uint32_t>(seed ^ (seed >> 32)) ^ (static_cast<uint32_t>(row) * 0x9E3779B1u) ^
                 (static_cast<uint32_t>(col) * 0x85EBCA77u) ^ (static_cast<uint32_t>(row >> 32) * 0xC2B2AE3Du);
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    const float u = static_cast<float>(h >> 8) * (1.0f / 16777216.0f);  // [0,1), 24 bits
    return u >= p;
}

// ---- activations (src/models/two_tower.py:77-86) ----
__device__ __forceinline__ float act_fwd(int act, float z) {
    switch (act) {
        case RT_ACT_RELU: return z > 0.f ? z : 0.f;
        case RT_ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case RT_ACT_LEAKY_RELU: return z > 0.f ? z : 0.1f * z;
        case RT_ACT_TANH: return tanhf(z);
        case RT_ACT_SIGMOID: return 1.f / (1.f + expf(-z));
        default: return z;
    }
}
// ReLU / LeakyReLU(0.1) / identity as ONE select (no per-element branch):
// z > 0 ? z : slope * z
__host__ __device__ __forceinline__ bool act_is_piecewise_linear(int act) {
    return act == RT_ACT_RELU || act == RT_ACT_LEAKY_RELU || act == RT_ACT_NONE;
}
__host__ __device__ __forceinline__ float act_slope(int act) {
    return act == RT_ACT_RELU ? 0.f : act == RT_ACT_LEAKY_RELU ? 0.1f : 1.f;
}
__device__ __forceinline__ float act_pwl(float slope, float z) { return z > 0.f ? z : slope * z; }

// d act / dz evaluated at z
__device__ __forceinline__ float act_bwd(int act, float z) {
    switch (act) {
        case RT_ACT_RELU: return z > 0.f ? 1.f : 0.f;
        case RT_ACT_GELU: {
            const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
            const float pdf = 0.39894228040143268f * expf(-0.5f * z * z);
            return cdf + z * pdf;
        }
        case RT_ACT_LEAKY_RELU: return z > 0.f ? 1.f : 0.1f;
        case RT_ACT_TANH: { const float t = tanhf(z); return 1.f - t * t; }
        case RT_ACT_SIGMOID: { const float s = 1.f / (1.f + expf(-z)); return s * (1.f - s); }
        default: return 1.f;
    }
}

// Code-size-aware forms for unrolled hot loops: piecewise-linear activations
// (ReLU / LeakyReLU / identity) inline as one select, the transcendental ones
// through an out-of-line call, so dozens of unrolled call sites do not inline
// erf/tanh/exp bodies (the instruction cache is shared by the CU pair)
__device__ __noinline__ float act_fwd_call(int act, float z) { return act_fwd(act, z); }
__device__ __noinline__ float act_bwd_call(int act, float z) { return act_bwd(act, z); }
__device__ __forceinline__ float act_eval(int act, float z) {
    return act_is_piecewise_linear(act) ? act_pwl(act_slope(act), z) : act_fwd_call(act, z);
}
__device__ __forceinline__ float act_grad_eval(int act, float z) {
    return act_is_piecewise_linear(act) ? (z > 0.f ? 1.f : act_slope(act)) : act_bwd_call(act, z);
}

// ---- (score, id) ordering: a better than b ⇔ score desc, then id asc ----
// ids are carried as uint32 local indices inside kernels; 0xFFFFFFFF = empty.
__device__ __forceinline__ bool better(float sa, uint32_t ia, float sb, uint32_t ib) {
    return sa > sb || (sa == sb && ia < ib);
}

constexpr uint32_t kEmptyId = 0xFFFFFFFFu;

}  // namespace rt
