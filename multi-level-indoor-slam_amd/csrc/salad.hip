// SALAD aggregation head on gfx950 -- the native branch of SALAD
// (place_recognition.py:357-368, 380-391), i.e. serizba/salad's SALAD aggregator over
// the DINOv2 ViT-B/14 final-LayerNorm tokens (oracle/salad.py restates it):
//
//   GEMM 1 (mlg_gemm_bias_relu_bf16): tokens [B*T, 768] -> relu(cluster_features.0 |
//          score.0) bf16 [B*T, 1024]
//   GEMM 2 (mlg_gemm_bias_f32_ld):    -> f32 [B*T, 256]: cols 0..127 cluster features
//          (cluster_features.3), 128..191 cluster scores (score.3), 192..255 zero
//          (the two 512 -> 128 / 64 layers as one block-diagonal K = 1024 weight)
//   k_salad_head (this file), one workgroup per frame:
//     token MLP on the CLS row (768 -> 512 relu -> 256, f32 weights),
//     the [65, n] score matrix with the dust-bin row resident in LDS (n <= 544),
//     3 log-domain Sinkhorn iterations (u over rows, v over columns, accurate expf /
//     logf log-sum-exp with the max shift, as torch.logsumexp), p = exp(log P - norm),
//     aggregation sum_n f[n, l] p[c, n] over the frame's tokens, per-cluster and global
//     L2 normalisation, output [256 token | 128 x 64 l-major] float32.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SL_C = 64;     // clusters
constexpr int SL_L = 128;    // cluster_dim
constexpr int SL_TOK = 256;  // token_dim
constexpr int SL_HID = 512;
constexpr int SL_NMAX = 544;  // patch tokens per frame held in LDS (322 x 322: 529)
constexpr int SL_THREADS = 512;
constexpr int SL_WAVES = SL_THREADS / 64;

// One output row of a Linear held by a wave: lanes stride K (coalesced), shuffle sum.
__device__ __forceinline__ float wave_row_dot(const float* __restrict__ w, const float* x, int K, int lane) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += w[k] * x[k];
    return wave_sum(s);
}

__global__ __launch_bounds__(SL_THREADS) void k_salad_head(const bf16_t* __restrict__ xn, const float* __restrict__ Y,
                                                          int T, const float* __restrict__ wt1,
                                                          const float* __restrict__ bt1, const float* __restrict__ wt2,
                                                          const float* __restrict__ bt2, float dust,
                                                          float* __restrict__ desc) {
    // LDS: the score / plan matrix [65][NS], then (after the aggregation) the normalised
    // aggregate [128][64] in its first 32 KB
    __shared__ float mat[(SL_C + 1) * SL_NMAX];
    __shared__ float u[SL_C + 1], v[SL_NMAX];
    __shared__ float tok[768], hid[SL_HID], tt[SL_TOK];
    __shared__ float cnorm[SL_C];
    __shared__ float red[SL_WAVES];

    const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n = T - 1;
    const int NS = n | 1;  // odd row stride: column-parallel reads are bank-conflict free
    const size_t row0 = (size_t)b * T;

    // ---- token MLP: t -> relu(W1 t + b1) -> W2 h + b2 (SALAD.token_features)
    for (int k = tid; k < 768; k += SL_THREADS) tok[k] = bf16_to_f32(xn[row0 * 768 + k]);
    __syncthreads();
    for (int j = wave; j < SL_HID; j += SL_WAVES) {
        const float s = wave_row_dot(wt1 + (size_t)j * 768, tok, 768, lane);
        if (lane == 0) hid[j] = fmaxf(s + bt1[j], 0.f);
    }
    __syncthreads();
    for (int j = wave; j < SL_TOK; j += SL_WAVES) {
        const float s = wave_row_dot(wt2 + (size_t)j * SL_HID, hid, SL_HID, lane);
        if (lane == 0) tt[j] = s + bt2[j];
    }

    // ---- score matrix [64 clusters | dust-bin row][n tokens]
    for (int e = tid; e < SL_C * n; e += SL_THREADS) {
        const int c = e & (SL_C - 1), j = e >> 6;
        mat[c * NS + j] = Y[(row0 + 1 + j) * 256 + 128 + c];
    }
    for (int j = tid; j < n; j += SL_THREADS) {
        mat[SL_C * NS + j] = dust;
        v[j] = 0.f;
    }
    __syncthreads();

    // log-marginals: norm = -log(n + m); the dust-bin row adds log(n - m) (float32 adds)
    const float norm = -(float)log((double)(n + SL_C));
    const float la_bin = norm + (float)log((double)(n - SL_C));

    for (int it = 0; it < 3; ++it) {
        // u_i = log a_i - logsumexp_j(M_ij + v_j): one wave per row
        for (int i = wave; i <= SL_C; i += SL_WAVES) {
            const float* r = mat + i * NS;
            float mx = -INFINITY;
            for (int j = lane; j < n; j += 64) mx = fmaxf(mx, r[j] + v[j]);
            mx = wave_max(mx);
            float s = 0.f;
            for (int j = lane; j < n; j += 64) s += expf((r[j] + v[j]) - mx);
            s = wave_sum(s);
            if (lane == 0) u[i] = (i == SL_C ? la_bin : norm) - (logf(s) + mx);
        }
        __syncthreads();
        // v_j = log b_j - logsumexp_i(M_ij + u_i): one thread per column
        for (int j = tid; j < n; j += SL_THREADS) {
            float mx = -INFINITY;
            for (int i = 0; i <= SL_C; ++i) mx = fmaxf(mx, mat[i * NS + j] + u[i]);
            float s = 0.f;
            for (int i = 0; i <= SL_C; ++i) s += expf((mat[i * NS + j] + u[i]) - mx);
            v[j] = norm - (logf(s) + mx);
        }
        __syncthreads();
    }
    // p = exp(M + u + v - norm), dust-bin row dropped
    for (int e = tid; e < SL_C * n; e += SL_THREADS) {
        const int c = e / n, j = e - c * n;
        float* m = mat + c * NS + j;
        *m = expf(((*m + u[c]) + v[j]) - norm);
    }
    __syncthreads();

    // ---- aggregation: agg[l][c] = sum_n f[n][l] p[c][n]; thread = (l, 16 clusters)
    const int l = tid & (SL_L - 1), cg = (tid >> 7) * 16;
    float acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    const float* f = Y + (row0 + 1) * 256 + l;
    for (int j = 0; j < n; ++j) {
        const float fv = f[(size_t)j * 256];
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] += fv * mat[(cg + q) * NS + j];
    }
    __syncthreads();  // every plan read done: the aggregate reuses the front of `mat`
#pragma unroll
    for (int q = 0; q < 16; ++q) mat[l * SL_C + cg + q] = acc[q];
    __syncthreads();
    // per-cluster L2 norm over l (F.normalize(dim=1), eps 1e-12)
    if (tid < SL_C) {
        float s = 0.f;
        for (int ll = 0; ll < SL_L; ++ll) s += mat[ll * SL_C + tid] * mat[ll * SL_C + tid];
        cnorm[tid] = fmaxf(sqrtf(s), 1e-12f);
    }
    __syncthreads();
    for (int e = tid; e < SL_L * SL_C; e += SL_THREADS) mat[e] = mat[e] / cnorm[e & (SL_C - 1)];
    // token part normalised the same way
    float st = 0.f;
    for (int j = tid; j < SL_TOK; j += SL_THREADS) st += tt[j] * tt[j];
    st = wave_sum(st);
    if (lane == 0) red[wave] = st;
    __syncthreads();
    float tn = 0.f;
    for (int w = 0; w < SL_WAVES; ++w) tn += red[w];
    tn = fmaxf(sqrtf(tn), 1e-12f);
    // global L2 norm of [t / |t|, agg]
    float sq = 0.f;
    for (int e = tid; e < SL_L * SL_C; e += SL_THREADS) sq += mat[e] * mat[e];
    for (int j = tid; j < SL_TOK; j += SL_THREADS) sq += (tt[j] / tn) * (tt[j] / tn);
    sq = wave_sum(sq);
    __syncthreads();
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    float tot = 0.f;
    for (int w = 0; w < SL_WAVES; ++w) tot += red[w];
    tot = fmaxf(sqrtf(tot), 1e-12f);
    float* o = desc + (size_t)b * (SL_TOK + SL_L * SL_C);
    for (int j = tid; j < SL_TOK; j += SL_THREADS) o[j] = (tt[j] / tn) / tot;
    for (int e = tid; e < SL_L * SL_C; e += SL_THREADS) o[SL_TOK + e] = mat[e] / tot;
}

}  // namespace

int mlg_salad_head(const bf16_t* xn, const float* Y, int B, int T, const float* wt1, const float* bt1,
                   const float* wt2, const float* bt2, float dust, float* desc, hipStream_t s) {
    const int n = T - 1;
    if (B <= 0 || n <= SL_C || (n | 1) > SL_NMAX) return MLG_EINVAL;  // rows are (n | 1) apart in LDS
    hipLaunchKernelGGL(k_salad_head, dim3(B), dim3(SL_THREADS), 0, s, xn, Y, T, wt1, bt1, wt2, bt2, dust, desc);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
