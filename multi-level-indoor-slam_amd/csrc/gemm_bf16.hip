// bf16 "NT" GEMM for the ViT-B/14 projections with fused epilogues (gfx950).
//
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] )
//
// A: activations, bf16 row-major [M, K]; W: nn.Linear weight, bf16 row-major [N, K].
// Both operands are K-contiguous, which is exactly what the 16x16x32 bf16 MFMA
// fragments want (8 consecutive k per lane).  The product is computed transposed
// (D = W . A^T per 16x16 tile) so that each lane ends up owning 4 consecutive output
// columns of one token row: epilogue stores are 8-byte bf16 / 16-byte f32 vectors.
//
// Tile 128 x 128 x 64, 256 threads (2 x 2 waves of 64 x 64), register-staged double
// buffer in LDS (64 KiB -> 2 workgroups per CU), st_16x32-style XOR swizzle
// (chunk ^ (row >> 1) & 7) that makes every ds_read_b128 fragment read conflict-free,
// XCD-aware bijective block remap so the N-tiles of one M-panel share an L2.
//
// Requirements (checked by the host launcher): K % 64 == 0, N % 128 == 0,
// 16-byte aligned A / W rows.  M is arbitrary (rows >= M are clamped on load and
// masked on store).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // one operand tile, 16 KiB

__device__ __forceinline__ int swz_off(int row, int chunk) {
    return row * (BK * 2) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// ------------------------------------------------------------------ epilogues
struct EpiF32 {  // plain f32 store (testing)
    float* C; int ldc;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        *reinterpret_cast<float4*>(C + (size_t)m * ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

struct EpiBiasBF16 {  // y = acc + b  -> bf16
    bf16_t* C; int ldc; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        uint2 o;
        o.x = pack_bf16x2(v[0] + b.x, v[1] + b.y);
        o.y = pack_bf16x2(v[2] + b.z, v[3] + b.w);
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = o;
    }
};

// nn.GELU() (exact, erf form).  erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7,
// far below the bf16 rounding of the output): one v_rcp, one v_exp, five FMAs instead
// of the ~30-instruction libm erff that made the fc1 epilogue VALU-bound.
__device__ __forceinline__ float erf_fast(float x) {
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float y = 1.0f - p * t * __expf(-ax * ax);
    return copysignf(y, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

struct EpiBiasGeluBF16 {  // y = gelu(acc + b) -> bf16   (mlp.fc1 + nn.GELU())
    bf16_t* C; int ldc; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        uint2 o;
        o.x = pack_bf16x2(gelu_erf(v[0] + b.x), gelu_erf(v[1] + b.y));
        o.y = pack_bf16x2(gelu_erf(v[2] + b.z), gelu_erf(v[3] + b.w));
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = o;
    }
};

struct EpiResidual {  // X += gamma * (acc + b)   (attn.proj / mlp.fc2 + LayerScale + residual)
    float* X; int ldx; const float* bias; const float* gamma;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        float4* p = reinterpret_cast<float4*>(X + (size_t)m * ldx + n);
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const float4 g = *reinterpret_cast<const float4*>(gamma + n);
        float4 x = *p;
        x.x += g.x * (v[0] + b.x);
        x.y += g.y * (v[1] + b.y);
        x.z += g.z * (v[2] + b.z);
        x.w += g.w * (v[3] + b.w);
        *p = x;
    }
};

struct EpiQKV {  // qkv -> Q, K bf16 [B, 12, Tpad, 64] and V^T bf16 [B, 12, 64, Tpad]
    bf16_t* Q; bf16_t* K; bf16_t* Vt; const float* bias; int T, Tpad;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const int bi = m / T, t = m - bi * T;
        const int which = n / 768, c = n - which * 768, h = c >> 6, d = c & 63;
        const size_t head = (size_t)bi * 12 + h;
        if (which < 2) {
            uint2 o;
            o.x = pack_bf16x2(v[0] + b.x, v[1] + b.y);
            o.y = pack_bf16x2(v[2] + b.z, v[3] + b.w);
            *reinterpret_cast<uint2*>((which == 0 ? Q : K) + (head * Tpad + t) * 64 + d) = o;
        } else {  // transposed so attention streams V^T rows (key-contiguous)
            bf16_t* p = Vt + (head * 64 + d) * Tpad + t;
            p[0] = f32_to_bf16(v[0] + b.x);
            p[Tpad] = f32_to_bf16(v[1] + b.y);
            p[2 * Tpad] = f32_to_bf16(v[2] + b.z);
            p[3 * Tpad] = f32_to_bf16(v[3] + b.w);
        }
    }
};

struct EpiPatch {  // patch tokens: X[b, 1 + p, :] = acc + b + pos[1 + p]
    float* X; const float* bias; const float* pos; int P;  // P = patches per image
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const int bi = m / P, p = m - bi * P;
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const float4 q = *reinterpret_cast<const float4*>(pos + (size_t)(1 + p) * 768 + n);
        *reinterpret_cast<float4*>(X + ((size_t)bi * (P + 1) + 1 + p) * 768 + n) =
            make_float4(v[0] + b.x + q.x, v[1] + b.y + q.y, v[2] + b.z + q.z, v[3] + b.w + q.w);
    }
};

// ---------------------------------------------------------------------- kernel
template <class Epi>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, Epi epi) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / BN, nM = (M + BM - 1) / BM, nwg = nN * nM;
    // XCD-aware bijective remap: hardware blocks b, b+8, ... (one XCD) get consecutive
    // logical ids, so the N-tiles of an M-panel run on one XCD and share its L2.
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    const int mt = wgid / nN, nt = wgid - mt * nN;
    const int m0 = mt * BM, n0 = nt * BN;

    // staging: 1024 16-B chunks per operand tile, 4 per thread (rows tid>>3 + 32 i)
    const int srow = tid >> 3, sch = tid & 7;
    const bf16_t* pa = A + (size_t)min(m0 + srow, M - 1) * lda + sch * 8;
    const bf16_t* pw = W + (size_t)(n0 + srow) * ldw + sch * 8;
    const size_t a32 = (size_t)lda * 32, w32 = (size_t)ldw * 32;
    // rows >= M are clamped to M - 1 (their products are never stored)
    const int ar1 = min(m0 + srow + 32, M - 1) - min(m0 + srow, M - 1);
    const int ar2 = min(m0 + srow + 64, M - 1) - min(m0 + srow, M - 1);
    const int ar3 = min(m0 + srow + 96, M - 1) - min(m0 + srow, M - 1);
    const int so0 = swz_off(srow, sch), so1 = swz_off(srow + 32, sch);
    const int so2 = swz_off(srow + 64, sch), so3 = swz_off(srow + 96, sch);
    uint4 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define GEMM_GLOAD(k0)                                                              \
    {                                                                               \
        ra0 = *reinterpret_cast<const uint4*>(pa + (k0));                           \
        ra1 = *reinterpret_cast<const uint4*>(pa + (size_t)ar1 * lda + (k0));       \
        ra2 = *reinterpret_cast<const uint4*>(pa + (size_t)ar2 * lda + (k0));       \
        ra3 = *reinterpret_cast<const uint4*>(pa + (size_t)ar3 * lda + (k0));       \
        rw0 = *reinterpret_cast<const uint4*>(pw + (k0));                           \
        rw1 = *reinterpret_cast<const uint4*>(pw + w32 + (k0));                     \
        rw2 = *reinterpret_cast<const uint4*>(pw + 2 * w32 + (k0));                 \
        rw3 = *reinterpret_cast<const uint4*>(pw + 3 * w32 + (k0));                 \
    }
#define GEMM_LSTORE(buf)                                                            \
    {                                                                               \
        char* b_ = smem + (buf) * 2 * TILE_BYTES;                                   \
        *reinterpret_cast<uint4*>(b_ + so0) = ra0;                                  \
        *reinterpret_cast<uint4*>(b_ + so1) = ra1;                                  \
        *reinterpret_cast<uint4*>(b_ + so2) = ra2;                                  \
        *reinterpret_cast<uint4*>(b_ + so3) = ra3;                                  \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so0) = rw0;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so1) = rw1;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so2) = rw2;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so3) = rw3;                     \
    }
    (void)a32;

    const int wn = wave >> 1, wm = wave & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    GEMM_GLOAD(0);
    GEMM_LSTORE(0);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) { GEMM_GLOAD((kt + 1) * BK); }
        const char* base = smem + cur * 2 * TILE_BYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[4], wf[4];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wm * 64 + j * 16 + (lane & 15);
                af[j] = *reinterpret_cast<const bf16x8*>(base + swz_off(row, ch));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = wn * 64 + i * 16 + (lane & 15);
                wf[i] = *reinterpret_cast<const bf16x8*>(base + TILE_BYTES + swz_off(row, ch));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) { GEMM_LSTORE(cur ^ 1); }
        __syncthreads();
        cur ^= 1;
    }

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
            const int m = m0 + wm * 64 + j * 16 + (lane & 15);
            if (m < M) epi(m, n, acc[i][j]);
        }
#undef GEMM_GLOAD
#undef GEMM_LSTORE
}

// ------------------------------------------------------------- kernel v2
// 128 x 256 x 64 tile, 512 threads = 8 waves (2 along M x 4 along N, 64 x 64 each),
// three LDS stages filled by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction), K-tile t+2 prefetched while t is computed.  The XOR swizzle
// moves to the per-lane SOURCE address (the DMA writes lane-linear); fragment reads
// apply the same involution.  Waits are counted (s_waitcnt vmcnt(6) = the six DMAs of
// the newest tile stay in flight across the raw s_barrier); each stage is its own
// __shared__ object and the loop is unrolled by 3 so stage addresses are constants.
namespace v2 {
constexpr int BM = 128, BN = 256, BK = 64;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;  // 48 KiB
typedef __attribute__((address_space(3))) char lds_char;

// LDS byte address of a __shared__ object (the value M0 carries for LDS-DMA).
__device__ __forceinline__ unsigned lds_addr(char* p) {
    return (unsigned)(uintptr_t)(lds_char*)p;
}

// One global_load_lds_dwordx4: 16 B per lane from `g` into LDS [m0 + 16 * lane].
// Issued through inline asm so hipcc's waitcnt pass does not conservatively drain
// vmcnt(0) before every fragment read of the other stages; all waits on these DMAs
// are the explicit counted s_waitcnt vmcnt of the pipeline.
__device__ __forceinline__ void dma16(const void* g, unsigned m0) {
    asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

template <class Epi>
__global__ __launch_bounds__(512, 1) void k_gemm(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, int M,
                                                 int N, int K, int lda, int ldw, Epi epi) {
    __shared__ __attribute__((aligned(16))) char st0[STAGE];
    __shared__ __attribute__((aligned(16))) char st1[STAGE];
    __shared__ __attribute__((aligned(16))) char st2[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / BN, nM = (M + BM - 1) / BM, nwg = nN * nM;
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    const int mt = wgid / nN, nt = wgid - mt * nN;
    const int m0 = mt * BM, n0 = nt * BN;

    // DMA sources: wave w fills A row-groups 2w, 2w+1 and B row-groups 4w .. 4w+3 (8 rows each)
    const int lr = lane >> 3, lp = lane & 7;
    int ra = (2 * wave) * 8 + lr;
    const bf16_t* pa0 = A + (size_t)min(m0 + ra, M - 1) * lda + ((lp ^ ((ra >> 1) & 7)) * 8);
    ra += 8;
    const bf16_t* pa1 = A + (size_t)min(m0 + ra, M - 1) * lda + ((lp ^ ((ra >> 1) & 7)) * 8);
    int rb = (4 * wave) * 8 + lr;
    const bf16_t* pb0 = W + (size_t)(n0 + rb) * ldw + ((lp ^ ((rb >> 1) & 7)) * 8);
    rb += 8;
    const bf16_t* pb1 = W + (size_t)(n0 + rb) * ldw + ((lp ^ ((rb >> 1) & 7)) * 8);
    rb += 8;
    const bf16_t* pb2 = W + (size_t)(n0 + rb) * ldw + ((lp ^ ((rb >> 1) & 7)) * 8);
    rb += 8;
    const bf16_t* pb3 = W + (size_t)(n0 + rb) * ldw + ((lp ^ ((rb >> 1) & 7)) * 8);
    const int da = (2 * wave) * 1024, db = A_BYTES + (4 * wave) * 1024;

#define V2_ISSUE(ST, k0)                                                                                   \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST);                                                                  \
        dma16(pa0 + (k0), b_ + da);                                                                        \
        dma16(pa1 + (k0), b_ + da + 1024);                                                                 \
        dma16(pb0 + (k0), b_ + db);                                                                        \
        dma16(pb1 + (k0), b_ + db + 1024);                                                                 \
        dma16(pb2 + (k0), b_ + db + 2048);                                                                 \
        dma16(pb3 + (k0), b_ + db + 3072);                                                                 \
    }

    const int wm = wave & 1, wn = wave >> 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define V2_COMPUTE(ST)                                                                                     \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                        \
        bf16x8 af[4], wf[4];                                                                               \
        const int ch = s * 4 + (lane >> 4);                                                                \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                    \
            const int row = wm * 64 + j * 16 + (lane & 15);                                                \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + swz_off(row, ch));                             \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                    \
            const int row = wn * 64 + i * 16 + (lane & 15);                                                \
            wf[i] = *reinterpret_cast<const bf16x8*>((ST) + A_BYTES + swz_off(row, ch));                   \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j)        \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);         \
    }

    // s_waitcnt encodings (gfx9): vmcnt(6) = 0xF76, vmcnt(0) = 0xF70 (lgkm/exp untouched).
    // Every step issues its DMA unconditionally (past the last K-tile it re-reads the
    // last tile into a stage that is never read again) so the waitcnt pass sees the
    // same pending-DMA state on every path and never falls back to vmcnt(0).
#define V2_STEP(TT, CUR, NXT)                                                                              \
    {                                                                                                      \
        V2_ISSUE(NXT, min((TT) + 2, nk - 1) * BK);                                                         \
        V2_COMPUTE(CUR);                                                                                   \
        __builtin_amdgcn_s_waitcnt(0xF76);                                                                 \
        __builtin_amdgcn_s_barrier();                                                                      \
    }

    const int nk = K / BK;  // multiple of 3 (checked by the launcher)
    V2_ISSUE(st0, 0);
    V2_ISSUE(st1, BK);
    __builtin_amdgcn_s_waitcnt(0xF76);
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; t += 3) {
        V2_STEP(t, st0, st2)
        V2_STEP(t + 1, st1, st0)
        V2_STEP(t + 2, st2, st1)
    }
    __builtin_amdgcn_s_waitcnt(0xF70);  // no DMA may still be writing LDS when the block retires
#undef V2_STEP
#undef V2_COMPUTE
#undef V2_ISSUE

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
            const int m = m0 + wm * 64 + j * 16 + (lane & 15);
            if (m < M) epi(m, n, acc[i][j]);
        }
}
}  // namespace v2

int g_variant = 2;  // 1: 128x128 register-staged, 2: 128x256 3-stage LDS-DMA

template <class Epi>
int launch(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, Epi epi, hipStream_t s,
           int variant = -1) {
    if (variant < 0) variant = g_variant;
    if (M <= 0 || N <= 0 || K <= 0 || (K % BK) || (lda % 8) || (ldw % 8) || lda < K || ldw < K)
        return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return MLG_EINVAL;
    if (variant == 2 && N % v2::BN == 0 && (K / BK) % 3 == 0) {
        const long nwg = (long)(N / v2::BN) * ((M + v2::BM - 1) / v2::BM);
        hipLaunchKernelGGL(v2::k_gemm<Epi>, dim3((unsigned)nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, epi);
    } else {
        if (N % BN) return MLG_EINVAL;
        const long nwg = (long)(N / BN) * ((M + BM - 1) / BM);
        hipLaunchKernelGGL(k_gemm_nt<Epi>, dim3((unsigned)nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, epi);
    }
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

}  // namespace

int mlg_gemm_f32out(const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiF32{C, N}, s);
}
int mlg_gemm_f32out_variant(int variant, const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K,
                            hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiF32{C, N}, s, variant);
}
int mlg_gemm_set_variant(int variant) {
    if (variant != 1 && variant != 2) return MLG_EINVAL;
    g_variant = variant;
    return MLG_OK;
}
int mlg_gemm_bias_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                       hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiBiasBF16{C, N, bias}, s);
}
int mlg_gemm_bias_gelu_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                            hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiBiasGeluBF16{C, N, bias}, s);
}
int mlg_gemm_residual(const bf16_t* A, const bf16_t* W, const float* bias, const float* gamma, float* X, int M,
                      int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiResidual{X, N, bias, gamma}, s);
}
int mlg_gemm_qkv(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* Q, bf16_t* Kh, bf16_t* V, int M,
                 int T, int Tpad, hipStream_t s) {
    if (M % T) return MLG_EINVAL;
    return launch(A, W, M, 3 * 768, 768, 768, 768, EpiQKV{Q, Kh, V, bias, T, Tpad}, s);
}
int mlg_gemm_patch(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, float* X, int M, int P,
                   int Kpad, hipStream_t s) {
    if (M % P) return MLG_EINVAL;
    return launch(A, W, M, 768, Kpad, Kpad, Kpad, EpiPatch{X, bias, pos, P}, s);
}
