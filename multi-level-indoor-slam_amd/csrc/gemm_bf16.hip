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

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

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

template <class Epi>
int launch(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, Epi epi, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || (N % BN) || (K % BK) || (lda % 8) || (ldw % 8) || lda < K || ldw < K)
        return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return MLG_EINVAL;
    const long nwg = (long)(N / BN) * ((M + BM - 1) / BM);
    hipLaunchKernelGGL(k_gemm_nt<Epi>, dim3((unsigned)nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, epi);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

}  // namespace

int mlg_gemm_f32out(const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiF32{C, N}, s);
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
