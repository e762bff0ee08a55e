// ResNet-50 global descriptor: the MixVPR / SALAD fallback of the reference
// (place_recognition.py:248-306; semantics in oracle/resnet.py).
//
//   BGR uint8 taken as RGB (no swap) -> Pillow bilinear antialiased resize to 224x224
//   (Resample.c fixed point, horizontal then vertical pass, uint8 in between; the
//   coefficient tables come from the host, computed exactly as Pillow does) -> /255 ->
//   ImageNet normalise -> resnet50 (eval BatchNorm folded into the convs) -> global
//   average pool -> 2048 floats, zero-padded / truncated to descriptor_dim.
//
// Layout: NHWC.  Stem 7x7/2 conv in f32 on the VALU (K = 147); 3x3/2 max-pool; every
// bottleneck conv is a bf16 MFMA GEMM (gemm_bf16.hip): 1x1 convs directly on the NHWC
// activation matrix, 3x3 convs on an im2col copy (k = tap * Cin + c).  The residual
// stream stays f32 (the conv3 epilogue adds bias + shortcut, applies ReLU and writes
// the bf16 copy the next GEMM reads).
#include <math.h>

#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int RN_S = 224;
constexpr int PB = 22;  // Pillow PRECISION_BITS

// Pillow ImagingResampleHorizontal_8bpc: out[b, y, xx, c] over all input rows.
__global__ void k_rn_resize_h(const uint8_t* __restrict__ frames, long frame_stride, int H, int W, int C,
                              const int* __restrict__ xmin, const int* __restrict__ xcnt,
                              const int* __restrict__ kk, int ksize, uint8_t* __restrict__ out, int B) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, y, xx)
    if (e >= (long)B * H * RN_S) return;
    const int xx = (int)(e % RN_S), y = (int)((e / RN_S) % H), b = (int)(e / ((long)RN_S * H));
    const uint8_t* row = frames + (size_t)b * frame_stride + (size_t)y * W * C;
    const int x0 = xmin[xx], n = xcnt[xx];
    const int* k = kk + xx * ksize;
    int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < n; ++x) {
        const uint8_t* p = row + (size_t)(x0 + x) * C;
        const int w = k[x];
        if (C >= 3) {
            s0 += p[0] * w;
            s1 += p[1] * w;
            s2 += p[2] * w;
        } else {
            s0 += p[0] * w;
        }
    }
    if (C < 3) s1 = s2 = s0;
    uint8_t* o = out + e * 3;
    o[0] = (uint8_t)min(max(s0 >> PB, 0), 255);
    o[1] = (uint8_t)min(max(s1 >> PB, 0), 255);
    o[2] = (uint8_t)min(max(s2 >> PB, 0), 255);
}

// vertical pass + ToTensor (/255) + Normalize -> f32 NHWC [B, 224, 224, 3]
__global__ void k_rn_resize_v(const uint8_t* __restrict__ tmp, int H, const int* __restrict__ ymin,
                              const int* __restrict__ ycnt, const int* __restrict__ kk, int ksize,
                              float* __restrict__ out, uint8_t* __restrict__ out_u8, int B) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, yy, x)
    if (e >= (long)B * RN_S * RN_S) return;
    const int x = (int)(e % RN_S), yy = (int)((e / RN_S) % RN_S), b = (int)(e / ((long)RN_S * RN_S));
    const int y0 = ymin[yy], n = ycnt[yy];
    const int* k = kk + yy * ksize;
    int s[3] = {1 << (PB - 1), 1 << (PB - 1), 1 << (PB - 1)};
    for (int y = 0; y < n; ++y) {
        const uint8_t* p = tmp + (((size_t)b * H + y0 + y) * RN_S + x) * 3;
        for (int c = 0; c < 3; ++c) s[c] += p[c] * k[y];
    }
    const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
    for (int c = 0; c < 3; ++c) {
        const int v = min(max(s[c] >> PB, 0), 255);
        if (out_u8) out_u8[e * 3 + c] = (uint8_t)v;  // parity entry: the resized image itself
        else out[e * 3 + c] = ((float)v / 255.0f - mean[c]) / stdv[c];
    }
}

// stem: 7x7 stride-2 pad-3 conv 3 -> 64 (folded BN) + ReLU, f32 math -> bf16 [B,112,112,64]
// and f32 copy is not needed (max-pool follows).  One thread per output pixel.
__global__ __launch_bounds__(256) void k_rn_stem(const float* __restrict__ img, const float* __restrict__ w,
                                                 const float* __restrict__ bias, bf16_t* __restrict__ out, int B) {
    __shared__ float sw[64 * 147];
    __shared__ float sb[64];
    for (int i = threadIdx.x; i < 64 * 147; i += 256) sw[i] = w[i];
    if (threadIdx.x < 64) sb[threadIdx.x] = bias[threadIdx.x];
    __syncthreads();
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)B * 112 * 112) return;
    const int x = (int)(e % 112), y = (int)((e / 112) % 112), b = (int)(e / (112 * 112));
    float acc[64];
#pragma unroll
    for (int co = 0; co < 64; ++co) acc[co] = 0.f;
    for (int ky = 0; ky < 7; ++ky)
        for (int kx = 0; kx < 7; ++kx) {
            const int yy = 2 * y - 3 + ky, xx = 2 * x - 3 + kx;
            const bool ok = yy >= 0 && yy < RN_S && xx >= 0 && xx < RN_S;
            const float* p = img + (((size_t)b * RN_S + (ok ? yy : 0)) * RN_S + (ok ? xx : 0)) * 3;
            for (int c = 0; c < 3; ++c) {
                const float v = ok ? p[c] : 0.f;
                const int k = (ky * 7 + kx) * 3 + c;
#pragma unroll
                for (int co = 0; co < 64; ++co) acc[co] += sw[co * 147 + k] * v;
            }
        }
    bf16_t* o = out + e * 64;
#pragma unroll
    for (int c0 = 0; c0 < 64; c0 += 8) {
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2)
            pk[j / 2] = pack_bf16x2(fmaxf(acc[c0 + j] + sb[c0 + j], 0.f), fmaxf(acc[c0 + j + 1] + sb[c0 + j + 1], 0.f));
        *reinterpret_cast<uint4*>(o + c0) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
}

// 3x3 stride-2 pad-1 max-pool, bf16 [B,112,112,64] -> f32 + bf16 [B,56,56,64]
__global__ void k_rn_maxpool(const bf16_t* __restrict__ in, float* __restrict__ outf, bf16_t* __restrict__ outb,
                             int B) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, y, x, c)
    if (e >= (long)B * 56 * 56 * 64) return;
    const int c = (int)(e % 64), x = (int)((e / 64) % 56), y = (int)((e / (64 * 56)) % 56), b = (int)(e / (64 * 56 * 56));
    float m = -INFINITY;
    for (int ky = 0; ky < 3; ++ky)
        for (int kx = 0; kx < 3; ++kx) {
            const int yy = 2 * y - 1 + ky, xx = 2 * x - 1 + kx;
            if (yy >= 0 && yy < 112 && xx >= 0 && xx < 112)
                m = fmaxf(m, bf16_to_f32(in[(((size_t)b * 112 + yy) * 112 + xx) * 64 + c]));
        }
    outf[e] = m;
    outb[e] = f32_to_bf16(m);
}

// im2col for a 3x3 pad-1 conv with stride s: [B*Ho*Wo, 9*C] bf16, k = tap * C + c
__global__ void k_rn_im2col(const bf16_t* __restrict__ in, int B, int H, int W, int C, int s,
                            bf16_t* __restrict__ out) {
    const int Ho = (H - 1) / s + 1, Wo = (W - 1) / s + 1;
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (row, tap, 8-channel chunk)
    const int cch = C / 8;
    if (e >= (long)B * Ho * Wo * 9 * cch) return;
    const int ch = (int)(e % cch), tap = (int)((e / cch) % 9);
    const long r = e / ((long)cch * 9);
    const int x = (int)(r % Wo), y = (int)((r / Wo) % Ho), b = (int)(r / ((long)Wo * Ho));
    const int yy = y * s - 1 + tap / 3, xx = x * s - 1 + tap % 3;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (yy >= 0 && yy < H && xx >= 0 && xx < W)
        v = *reinterpret_cast<const uint4*>(in + (((size_t)b * H + yy) * W + xx) * C + ch * 8);
    *reinterpret_cast<uint4*>(out + r * 9 * C + tap * C + ch * 8) = v;
}

// stride-2 subsample of a bf16 NHWC activation (the input of a strided 1x1 downsample)
__global__ void k_rn_subsample(const bf16_t* __restrict__ in, int B, int H, int W, int C, bf16_t* __restrict__ out) {
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, cch = C / 8;
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)B * Ho * Wo * cch) return;
    const int ch = (int)(e % cch);
    const long r = e / cch;
    const int x = (int)(r % Wo), y = (int)((r / Wo) % Ho), b = (int)(r / ((long)Wo * Ho));
    *reinterpret_cast<uint4*>(out + r * C + ch * 8) =
        *reinterpret_cast<const uint4*>(in + (((size_t)b * H + 2 * y) * W + 2 * x) * C + ch * 8);
}

// global average pool (f32 [B, HW, 2048]) -> desc [B, D] zero-padded / truncated
__global__ void k_rn_avgpool(const float* __restrict__ x, int B, int HW, int D, float* __restrict__ desc) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)B * D) return;
    const int c = (int)(e % D), b = (int)(e / D);
    float v = 0.f;
    if (c < 2048) {
        float s = 0.f;
        for (int i = 0; i < HW; ++i) s += x[((size_t)b * HW + i) * 2048 + c];
        v = s / (float)HW;
    }
    desc[e] = v;
}

// Pillow precompute_coeffs (bilinear, support 1) + normalize_coeffs_8bpc, host side.
struct Coeffs {
    int ksize = 0;
    std::vector<int> xmin, xcnt, kk;
};

Coeffs pillow_coeffs(int in_size, int out_size) {
    Coeffs c;
    const double scale = (double)(float)in_size / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * filterscale;
    c.ksize = (int)ceil(support) * 2 + 1;
    c.xmin.resize(out_size);
    c.xcnt.resize(out_size);
    c.kk.assign((size_t)out_size * c.ksize, 0);
    std::vector<double> k(c.ksize);
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = (xx + 0.5) * scale;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        double ww = 0.0;
        for (int x = 0; x < xmax; ++x) {
            double t = (x + xmin - center + 0.5) * ss;
            if (t < 0.0) t = -t;
            const double w = t < 1.0 ? 1.0 - t : 0.0;
            k[x] = w;
            ww += w;
        }
        for (int x = 0; x < xmax; ++x) {
            const double v = ww != 0.0 ? k[x] / ww : k[x];
            c.kk[(size_t)xx * c.ksize + x] = v < 0 ? (int)(-0.5 + v * (1 << PB)) : (int)(0.5 + v * (1 << PB));
        }
        c.xmin[xx] = xmin;
        c.xcnt[xx] = xmax;
    }
    return c;
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct RnLayout {
    size_t tables, tmp, img, stem, xf0, xf1, xb0, xb1, t1, t2, col, sub, total;
};

RnLayout rn_layout(int B, int H) {
    RnLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += a256(bytes);
        return r;
    };
    const size_t m56 = (size_t)B * 56 * 56;
    L.tables = take((size_t)4 * (2 * RN_S + RN_S * 64) * 2 + 4096);  // generous: two (xmin, xcnt, kk) sets
    L.tmp = take((size_t)B * H * RN_S * 3);
    L.img = take((size_t)B * RN_S * RN_S * 3 * 4);
    L.stem = take((size_t)B * 112 * 112 * 64 * 2);
    L.xf0 = take(m56 * 256 * 4);  // largest residual tensor: stage 1, 56x56x256
    L.xf1 = take(m56 * 256 * 4);
    L.xb0 = take(m56 * 256 * 2);
    L.xb1 = take(m56 * 256 * 2);
    L.t1 = take(m56 * 128 * 2);   // bottleneck conv1 out (<= 56x56x64 padded to 128, 28x28x128 ...)
    L.t2 = take(m56 * 128 * 2);   // conv2 out
    L.col = take(m56 * 9 * 64 * 2 > (size_t)B * 28 * 28 * 9 * 128 * 2 ? m56 * 9 * 64 * 2
                                                                          : (size_t)B * 28 * 28 * 9 * 128 * 2);
    L.sub = take((size_t)B * 28 * 28 * 256 * 2);
    L.total = o;
    return L;
}

// Tables per input size, never freed: pending async uploads keep reading them.
struct CoeffCache {
    std::mutex mu;
    std::map<int, Coeffs> by_size;
    const Coeffs& get(int in_size) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = by_size.find(in_size);
        if (it == by_size.end()) it = by_size.emplace(in_size, pillow_coeffs(in_size, RN_S)).first;
        return it->second;
    }
} g_coeffs;

}  // namespace

size_t mlg_resnet50_ws_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return rn_layout(B, H).total;
}

int mlg_resnet50_run(const mlg_rn_weights_i& w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                     int D, void* ws, size_t ws_bytes, float* desc, uint8_t* resized_u8, hipStream_t s) {
    if (B <= 0 || H <= 0 || W <= 0 || (C != 1 && C != 3 && C != 4) || D <= 0) return MLG_EINVAL;
    const RnLayout L = rn_layout(B, H);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* base = (char*)ws;
    const Coeffs& ch = g_coeffs.get(W);
    const Coeffs& cv = g_coeffs.get(H);
    int* tb = (int*)(base + L.tables);
    int* hx0 = tb;
    int* hxc = hx0 + RN_S;
    int* hkk = hxc + RN_S;
    int* vy0 = hkk + (size_t)RN_S * ch.ksize;
    int* vyc = vy0 + RN_S;
    int* vkk = vyc + RN_S;
    if ((size_t)((char*)(vkk + (size_t)RN_S * cv.ksize) - (char*)tb) > L.tmp - L.tables) return MLG_EINVAL;
    if (hipMemcpyAsync(hx0, ch.xmin.data(), RN_S * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(hxc, ch.xcnt.data(), RN_S * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(hkk, ch.kk.data(), ch.kk.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(vy0, cv.xmin.data(), RN_S * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(vyc, cv.xcnt.data(), RN_S * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(vkk, cv.kk.data(), cv.kk.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return MLG_EHIP;
    uint8_t* tmp = (uint8_t*)(base + L.tmp);
    float* img = (float*)(base + L.img);
    bf16_t* stem = (bf16_t*)(base + L.stem);
    float* xf[2] = {(float*)(base + L.xf0), (float*)(base + L.xf1)};
    bf16_t* xb[2] = {(bf16_t*)(base + L.xb0), (bf16_t*)(base + L.xb1)};
    bf16_t* t1 = (bf16_t*)(base + L.t1);
    bf16_t* t2 = (bf16_t*)(base + L.t2);
    bf16_t* col = (bf16_t*)(base + L.col);
    bf16_t* sub = (bf16_t*)(base + L.sub);

    const long nh = (long)B * H * RN_S;
    hipLaunchKernelGGL(k_rn_resize_h, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, s, frames, frame_stride, H, W,
                       C, hx0, hxc, hkk, ch.ksize, tmp, B);
    const long nv = (long)B * RN_S * RN_S;
    hipLaunchKernelGGL(k_rn_resize_v, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, tmp, H, vy0, vyc, vkk,
                       cv.ksize, img, resized_u8, B);
    if (resized_u8) {  // parity entry: stop after the resize
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    }
    const long ns = (long)B * 112 * 112;
    hipLaunchKernelGGL(k_rn_stem, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, img, w.stem_w, w.stem_b, stem,
                       B);
    const long np = (long)B * 56 * 56 * 64;
    hipLaunchKernelGGL(k_rn_maxpool, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, stem, xf[0], xb[0], B);
    MLG_LAUNCH_CHECK();

    int cur = 0, Hc = 56, Cc = 64, blk = 0;
    const int widths[4] = {64, 128, 256, 512}, nblocks[4] = {3, 4, 6, 3};
    for (int st = 0; st < 4; ++st) {
        const int width = widths[st], wpad = width < 128 ? 128 : width;
        for (int bi = 0; bi < nblocks[st]; ++bi, ++blk) {
            const mlg_rn_block_i& bw = w.blocks[blk];
            const int stride = (st > 0 && bi == 0) ? 2 : 1;
            const int Ho = (Hc - 1) / stride + 1;
            const int M_in = B * Hc * Hc, M_out = B * Ho * Ho;
            const int nxt = cur ^ 1;
            // conv1 1x1 (+BN, ReLU) at the input resolution
            int rc = mlg_gemm_bias_relu_bf16(xb[cur], Cc, bw.w1, bw.b1, t1, width, width, M_in, wpad, Cc, s);
            if (rc != MLG_OK) return rc;
            // conv2 3x3 / stride (+BN, ReLU) via im2col
            const long ni = (long)M_out * 9 * (width / 8);
            hipLaunchKernelGGL(k_rn_im2col, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, s, t1, B, Hc, Hc, width,
                               stride, col);
            MLG_LAUNCH_CHECK();
            rc = mlg_gemm_bias_relu_bf16(col, 9 * width, bw.w2, bw.b2, t2, width, width, M_out, wpad, 9 * width, s);
            if (rc != MLG_OK) return rc;
            // shortcut: downsample conv (+BN) into the next f32 stream, or identity in place
            float* res = xf[cur];
            if (bw.wd) {
                const bf16_t* src = xb[cur];
                if (stride == 2) {
                    const long nsb = (long)M_out * (Cc / 8);
                    hipLaunchKernelGGL(k_rn_subsample, dim3((unsigned)((nsb + 255) / 256)), dim3(256), 0, s, xb[cur],
                                       B, Hc, Hc, Cc, sub);
                    MLG_LAUNCH_CHECK();
                    src = sub;
                }
                rc = mlg_gemm_bias_f32_ld(src, Cc, bw.wd, bw.bd, xf[nxt], 4 * width, M_out, 4 * width, Cc, s);
                if (rc != MLG_OK) return rc;
                res = xf[nxt];
            }
            // conv3 1x1 (+BN) + shortcut + ReLU -> f32 stream and its bf16 copy
            float* outf = bw.wd ? xf[nxt] : xf[cur];
            bf16_t* outb = xb[nxt];
            rc = mlg_gemm_bias_add_relu(t2, width, bw.w3, bw.b3, res, outf, 4 * width, outb, M_out, 4 * width, width,
                                        s);
            if (rc != MLG_OK) return rc;
            if (bw.wd) {
                cur = nxt;
            } else {
                // f32 stream updated in place (xf[cur]); bf16 copy went to xb[nxt]
                std::swap(xb[cur], xb[nxt]);
            }
            Hc = Ho;
            Cc = 4 * width;
        }
    }
    const long nd = (long)B * D;
    hipLaunchKernelGGL(k_rn_avgpool, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, xf[cur], B, Hc * Hc, D,
                       desc);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
