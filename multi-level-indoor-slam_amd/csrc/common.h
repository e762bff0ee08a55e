// Shared device helpers for the mlgate HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bfloat16 bits
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // 16x16x32 / 32x32x16 A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define MLG_OK 0
#define MLG_EINVAL (-1)
#define MLG_EHIP (-2)
#define MLG_ENOMEM (-3)

#define MLG_LAUNCH_CHECK()                                     \
    do {                                                       \
        hipError_t e_ = hipGetLastError();                     \
        if (e_ != hipSuccess) return MLG_EHIP;                 \
    } while (0)

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
    return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16 (v_cvt_pk_bf16_f32; NaN stays NaN).
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
    return (bf16_t)(pack_bf16x2(f, 0.0f) & 0xffffu);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
