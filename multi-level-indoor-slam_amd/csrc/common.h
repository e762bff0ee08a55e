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

// LoFTR FPN merge: lat + bilinear(v00, v01, v10, v11) with explicit rounding (no FMA
// contraction), shared by k_lf_up_add (loftr.hip) and the fused lateral-conv epilogue
// EpiConvUp (gemm_bf16.hip), so the two forms give the same bits
__device__ __forceinline__ float lf_up_add1(float lat, float a, float b, float c, float d, float lx0, float lx1,
                                            float ly0, float ly1) {
    const float t0 = __fadd_rn(__fmul_rn(lx0, a), __fmul_rn(lx1, b));
    const float t1 = __fadd_rn(__fmul_rn(lx0, c), __fmul_rn(lx1, d));
    return __fadd_rn(lat, __fadd_rn(__fmul_rn(ly0, t0), __fmul_rn(ly1, t1)));
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
    return (bf16_t)(pack_bf16x2(f, 0.0f) & 0xffffu);
}

// Split-bf16 pairs (MLG_VIT_SPLIT): hi = bf16(x) (RNE), lo = bf16(x - hi); x - hi is exact
// in f32, so x = hi + lo to 2^-17 relative.  Four floats -> two packed bf16x2 each.
__device__ __forceinline__ void split_bf16x4(float a, float b, float c, float d, uint2& hi, uint2& lo) {
    hi.x = pack_bf16x2(a, b);
    hi.y = pack_bf16x2(c, d);
    lo.x = pack_bf16x2(a - __uint_as_float(hi.x << 16), b - __uint_as_float(hi.x & 0xffff0000u));
    lo.y = pack_bf16x2(c - __uint_as_float(hi.y << 16), d - __uint_as_float(hi.y & 0xffff0000u));
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

// LightGlue rotary factors, one float4 per (token row r, frequency pair p):
// (cos f, cos f + 1, sin f, sin f + 1), f = 2 p, laid out per 64-row tile as
// [Npad / 64][16 pairs][64 rows] -- a tile's factors are one contiguous 16 KiB block (one
// LDS-DMA stream), and the 32 rows a projection epilogue lane group reads for one pair
// are 512 contiguous bytes (a conflict-free ds_read_b128; profiles/r05c_lds_conflict_calibration.txt).
__host__ __device__ __forceinline__ size_t lg_fac4(size_t r, int p) {
    return ((r >> 6) * 16 + (size_t)p) * 64 + (r & 63);
}

// nn.GELU() (exact, erf form) as x * Phi(x) with Phi(x) = 0.5 + xc * P(2 xc^2 / 4.5^2 - 1),
// xc = clamp(x, -4.5, 4.5), P of degree 12 (a Chebyshev least-squares fit of
// (Phi(x) - 0.5) / x in the well-conditioned variable, evaluated by Horner in f32):
// |error| <= 1e-6 on [-4.5, 4.5], <= 3.4e-6 |x| beyond; on N(0, 1.3) inputs its bf16
// outputs differ from exact GELU's in 0.08 % of elements (A & S 7.1.26: 0.07 %, torch's
// own f32 GELU: 0.10 %).  No transcendental: pairs of calls pack into v_pk_fma_f32 (two
// scalar v_fma_f32 chains instead: the LightGlue block tail unchanged, the split ViT fc1
// epilogue 65 % slower and not bit-identical -- profiles/r05k_ab_gelu_scalar.txt).
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu_poly2(f32x2 x) {
    f32x2 xc;
    xc.x = __builtin_amdgcn_fmed3f(x.x, -4.5f, 4.5f);
    xc.y = __builtin_amdgcn_fmed3f(x.y, -4.5f, 4.5f);
    const f32x2 t = xc * xc * (2.0f / 20.25f) - 1.0f;
    f32x2 p = 0.000136977251f;
    p = p * t + -0.000375893549f;
    p = p * t + 0.000569374999f;
    p = p * t + -0.00130509574f;
    p = p * t + 0.00317945634f;
    p = p * t + -0.00628771959f;
    p = p * t + 0.0111988205f;
    p = p * t + -0.0185670499f;
    p = p * t + 0.0283403341f;
    p = p * t + -0.0401903689f;
    p = p * t + 0.0546963513f;
    p = p * t + -0.0771897957f;
    p = p * t + 0.156904995f;
    return x * (xc * p + 0.5f);
}
