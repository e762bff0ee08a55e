// Memory-bound ViT-B/14 ops around the GEMMs (gfx950): preprocessing + patch
// extraction, CLS rows, LayerNorm, and the fused final-LayerNorm + local-feature +
// GeM pooling of the CricaVPR descriptor.
#include "common.h"
#include "kernels.h"

namespace {

// ----------------------------------------------------------- preprocessing ---
// CricaVPR._preprocess (place_recognition.py:781-803) fused with the patch-embed
// im2col: cv2.resize INTER_LINEAR on uint8 (OpenCV fixed-point generic path:
// 11-bit weights, 128-bit vector vertical pass + scalar tail -- the same restatement
// as oracle/csrc/oracle.c), BGR/BGRA/gray -> RGB, float32 /255, float64
// (x - mean) / std, -> bf16 patch rows A[b*P + p, k], k = c*196 + ky*14 + kx
// (Conv2d weight order), zero for k in [588, Kpad).

__device__ __forceinline__ int16_t sat16(int v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

__device__ __forceinline__ void axis_lookup(int d, int ssize, int dsize, bool clamp, int& s0, int& s1, int& w0,
                                            int& w1) {
    const double scale = 1.0 / ((double)dsize / ssize);
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (clamp) {
        if (s < 0) { f = 0.f; s = 0; }
        if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
    }
    w0 = sat16((int)__builtin_rintf((1.f - f) * 2048.f));
    w1 = sat16((int)__builtin_rintf(f * 2048.f));
    s0 = min(max(s, 0), ssize - 1);
    s1 = min(max(s + 1, 0), ssize - 1);
}

__device__ __forceinline__ int resize_vec_end(int wb) {
    int x = 0;
    if (wb >= 16) x = ((wb - 16) / 16 + 1) * 16;
    while (x < wb - 8) x += 8;
    return x;
}

struct PrepParams {
    const uint8_t* img;  // [B, H, W, C]
    int H, W, C, S, grid, P, Kpad;
    int swap_rb;         // 1: BGR(A) -> RGB (CricaVPR); 0: channels fed as stored (AnyLoc, :495-505)
    long img_stride;     // bytes between images
    bf16_t* out;         // [B*P, Kpad], or [B*P, 2 Kpad] = [hi | lo] rows when split
    int split;           // MLG_VIT_SPLIT: split-bf16 pairs
};

__global__ __launch_bounds__(256) void k_preprocess_patches(PrepParams pp, int total_chunks) {
    __shared__ float lut[3][256];
    for (int i = threadIdx.x; i < 768; i += 256) {
        const int c = i >> 8, u = i & 255;
        const double mean = c == 0 ? 0.485 : (c == 1 ? 0.456 : 0.406);
        const double std = c == 0 ? 0.229 : (c == 1 ? 0.224 : 0.225);
        const float x = (float)u / 255.0f;
        lut[c][u] = (float)(((double)x - mean) / std);
    }
    __syncthreads();
    const int kchunks = pp.Kpad / 8;
    const int vend = resize_vec_end(pp.S * pp.C);
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total_chunks; idx += gridDim.x * 256) {
        const int row = idx / kchunks, kc = idx - row * kchunks;
        const int b = row / pp.P, p = row - b * pp.P;
        const int py = p / pp.grid, px = p - py * pp.grid;
        const uint8_t* src = pp.img + (size_t)b * pp.img_stride;
        float vals[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            float v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k = kc * 8 + e + u;
                float val = 0.f;
                if (k < 588) {
                    const int c = k / 196, rem = k - c * 196, ky = rem / 14, kx = rem - ky * 14;
                    const int y = py * 14 + ky, x = px * 14 + kx;
                    const int sc = pp.C == 1 ? 0 : (pp.swap_rb ? 2 - c : c);  // RGB c <- BGR(A) 2-c
                    int sx0, sx1, ax0, ax1, sy0, sy1, by0, by1;
                    axis_lookup(x, pp.W, pp.S, true, sx0, sx1, ax0, ax1);
                    axis_lookup(y, pp.H, pp.S, false, sy0, sy1, by0, by1);
                    const uint8_t* r0 = src + (size_t)sy0 * pp.W * pp.C;
                    const uint8_t* r1 = src + (size_t)sy1 * pp.W * pp.C;
                    const int h0 = r0[sx0 * pp.C + sc] * ax0 + r0[sx1 * pp.C + sc] * ax1;
                    const int h1 = r1[sx0 * pp.C + sc] * ax0 + r1[sx1 * pp.C + sc] * ax1;
                    int q;
                    if (x * pp.C + sc < vend) {  // universal-intrinsic vertical pass
                        const int a0 = sat16(h0 >> 4), a1 = sat16(h1 >> 4);
                        int t = (int16_t)(((a0 * by0) >> 16) + ((a1 * by1) >> 16));
                        q = (t + 2) >> 2;
                    } else {  // scalar tail
                        q = (h0 * by0 + h1 * by1 + (1 << 21)) >> 22;
                    }
                    q = min(max(q, 0), 255);
                    val = lut[c][q];
                }
                v2[u] = val;
            }
            vals[e] = v2[0];
            vals[e + 1] = v2[1];
        }
        if (pp.split) {
            uint2 h0, l0, h1, l1;
            split_bf16x4(vals[0], vals[1], vals[2], vals[3], h0, l0);
            split_bf16x4(vals[4], vals[5], vals[6], vals[7], h1, l1);
            bf16_t* o = pp.out + (size_t)row * 2 * pp.Kpad + kc * 8;
            *reinterpret_cast<uint4*>(o) = make_uint4(h0.x, h0.y, h1.x, h1.y);
            *reinterpret_cast<uint4*>(o + pp.Kpad) = make_uint4(l0.x, l0.y, l1.x, l1.y);
        } else {
            *reinterpret_cast<uint4*>(pp.out + (size_t)row * pp.Kpad + kc * 8) =
                make_uint4(pack_bf16x2(vals[0], vals[1]), pack_bf16x2(vals[2], vals[3]), pack_bf16x2(vals[4], vals[5]),
                           pack_bf16x2(vals[6], vals[7]));
        }
    }
}

// LayerNorm as split-bf16 pairs: rows of 1536, hi in columns 0..767, lo in 768..1535
__global__ __launch_bounds__(256) void k_layernorm_split(const float* __restrict__ X, const float* __restrict__ g,
                                                         const float* __restrict__ b, bf16_t* __restrict__ Y, int M);

// X[b, 0, :] = cls + pos[0]
__global__ void k_cls_rows(float* X, const float* cls, const float* pos, int T) {
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < 768; c += blockDim.x) X[(size_t)b * T * 768 + c] = cls[c] + pos[c];
}

// ---------------------------------------------------------------- LayerNorm ---
// torch.nn.LayerNorm(768, eps=1e-6): biased variance, one wave per token row.
__device__ __forceinline__ void ln_row(const float* x, const float* g, const float* bt, int lane, float4 (&y)[3]) {
    float4 v[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = *reinterpret_cast<const float4*>(x + i * 256 + lane * 4);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mean = wave_sum(s) * (1.0f / 768.0f);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
        q += (a * a + b * b) + (c * c + d * d);
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.0f / 768.0f) + 1e-6f);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float4 gg = *reinterpret_cast<const float4*>(g + i * 256 + lane * 4);
        const float4 bb = *reinterpret_cast<const float4*>(bt + i * 256 + lane * 4);
        y[i].x = (v[i].x - mean) * rstd * gg.x + bb.x;
        y[i].y = (v[i].y - mean) * rstd * gg.y + bb.y;
        y[i].z = (v[i].z - mean) * rstd * gg.z + bb.z;
        y[i].w = (v[i].w - mean) * rstd * gg.w + bb.w;
    }
}

__global__ __launch_bounds__(256) void k_layernorm_bf16(const float* __restrict__ X, const float* __restrict__ g,
                                                        const float* __restrict__ b, bf16_t* __restrict__ Y, int M) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float4 y[3];
    ln_row(X + (size_t)row * 768, g, b, lane, y);
#pragma unroll
    for (int i = 0; i < 3; ++i)
        *reinterpret_cast<uint2*>(Y + (size_t)row * 768 + i * 256 + lane * 4) =
            make_uint2(pack_bf16x2(y[i].x, y[i].y), pack_bf16x2(y[i].z, y[i].w));
}

__global__ __launch_bounds__(256) void k_layernorm_split(const float* __restrict__ X, const float* __restrict__ g,
                                                         const float* __restrict__ b, bf16_t* __restrict__ Y, int M) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float4 y[3];
    ln_row(X + (size_t)row * 768, g, b, lane, y);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        uint2 h, l;
        split_bf16x4(y[i].x, y[i].y, y[i].z, y[i].w, h, l);
        *reinterpret_cast<uint2*>(Y + (size_t)row * 1536 + i * 256 + lane * 4) = h;
        *reinterpret_cast<uint2*>(Y + (size_t)row * 1536 + 768 + i * 256 + lane * 4) = l;
    }
}

// Final norm + CricaVPR heads.  get_intermediate_layers strips CLS (token 0) and the
// CricaVPR code drops the first patch (token 1): tokens 2..T-1 are the local features
// [B, T-2, 768] (f32, extract_local_features) and GeM pools over exactly those.
// Block (b, chunk) normalises GEM_CHUNK tokens and writes per-chunk sums of
// clamp(x, 1e-6)^3; k_gem_finish reduces the chunks in a fixed order.
constexpr int GEM_CHUNKS = 8;

__global__ __launch_bounds__(256) void k_final_norm_gem(const float* __restrict__ X, const float* __restrict__ g,
                                                        const float* __restrict__ bt, float* __restrict__ local,
                                                        float* __restrict__ partial, int T, int mean_pool) {
    __shared__ float red[4][768];
    const int b = blockIdx.x, chunk = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int L = T - 2, per = (L + GEM_CHUNKS - 1) / GEM_CHUNKS;
    const int t0 = chunk * per, t1 = min(L, t0 + per);
    float acc[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = 0.f;
    for (int t = t0 + wave; t < t1; t += 4) {
        float4 y[3];
        ln_row(X + ((size_t)b * T + 2 + t) * 768, g, bt, lane, y);
        float* dst = local ? local + ((size_t)b * L + t) * 768 : nullptr;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (dst) *reinterpret_cast<float4*>(dst + i * 256 + lane * 4) = y[i];
            if (mean_pool) {  // AnyLoc: patch_features.mean(dim=1)
                acc[4 * i + 0] += y[i].x;
                acc[4 * i + 1] += y[i].y;
                acc[4 * i + 2] += y[i].z;
                acc[4 * i + 3] += y[i].w;
            } else {  // CricaVPR GeM p = 3: clamp(min=1e-6)^3
                const float c0 = fmaxf(y[i].x, 1e-6f), c1 = fmaxf(y[i].y, 1e-6f);
                const float c2 = fmaxf(y[i].z, 1e-6f), c3 = fmaxf(y[i].w, 1e-6f);
                acc[4 * i + 0] += c0 * c0 * c0;
                acc[4 * i + 1] += c1 * c1 * c1;
                acc[4 * i + 2] += c2 * c2 * c2;
                acc[4 * i + 3] += c3 * c3 * c3;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wave][i * 256 + lane * 4 + j] = acc[4 * i + j];
    __syncthreads();
    for (int c = threadIdx.x; c < 768; c += 256)
        partial[((size_t)b * GEM_CHUNKS + chunk) * 768 + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

__global__ void k_gem_finish(const float* __restrict__ partial, float* __restrict__ desc, int L, int mean_pool) {
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < 768; c += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < GEM_CHUNKS; ++k) s += partial[((size_t)b * GEM_CHUNKS + k) * 768 + c];
        desc[(size_t)b * 768 + c] = mean_pool ? s / (float)L : powf(s / (float)L, 1.0f / 3.0f);
    }
}

}  // namespace

int mlg_preprocess_patches(const uint8_t* img, int B, int H, int W, int C, long img_stride, int S, int Kpad,
                           int swap_rb, bf16_t* out, hipStream_t s, int split) {
    if (B <= 0 || H < 1 || W < 1 || !(C == 1 || C == 3 || C == 4) || S % 14 || Kpad < 588 || Kpad % 8)
        return MLG_EINVAL;
    PrepParams pp{img, H, W, C, S, S / 14, (S / 14) * (S / 14), Kpad, swap_rb, img_stride, out, split};
    const long total = (long)B * pp.P * (Kpad / 8);
    const int blocks = (int)std::min<long>((total + 255) / 256, 256L * 16);
    hipLaunchKernelGGL(k_preprocess_patches, dim3(blocks), dim3(256), 0, s, pp, (int)total);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_cls_rows(float* X, const float* cls, const float* pos, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(k_cls_rows, dim3(B), dim3(256), 0, s, X, cls, pos, T);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_layernorm_bf16(const float* X, const float* g, const float* b, bf16_t* Y, int M, hipStream_t s) {
    if (M <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_layernorm_bf16, dim3((M + 3) / 4), dim3(256), 0, s, X, g, b, Y, M);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_layernorm_split(const float* X, const float* g, const float* b, bf16_t* Y, int M, hipStream_t s) {
    if (M <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_layernorm_split, dim3((M + 3) / 4), dim3(256), 0, s, X, g, b, Y, M);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_final_norm_gem(const float* X, const float* g, const float* b, float* local, float* partial, float* desc,
                       int B, int T, int mean_pool, hipStream_t s) {
    if (B <= 0 || T < 3) return MLG_EINVAL;
    hipLaunchKernelGGL(k_final_norm_gem, dim3(B, GEM_CHUNKS), dim3(256), 0, s, X, g, b, local, partial, T, mean_pool);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gem_finish, dim3(B), dim3(256), 0, s, partial, desc, T - 2, mean_pool);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

size_t mlg_gem_partial_bytes(int B) { return (size_t)B * GEM_CHUNKS * 768 * sizeof(float); }
