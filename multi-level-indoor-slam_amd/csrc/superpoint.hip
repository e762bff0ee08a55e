// SuperPoint keypoints + descriptors for a batch of BGR keyframes (gfx950).
//
// Restates LightGlue's SuperPoint forward as called by the reference
// (geometric_verification.py:224-233, 263-312; semantics in oracle/superpoint.py):
// cv2 BGR2GRAY / 255 -> VGG encoder (3x3 convs + ReLU, 2x2 max-pools) -> detector
// head (softmax over 65, depth-to-space) -> simple_nms(4) -> border 4 -> threshold
// -> top-k -> descriptor head (L2-normalised) sampled bilinearly at the keypoints.
//
// Any H, W >= 16: conv1a / conv1b run at full resolution, the 2x2 pools round down,
// and the score / NMS / border / descriptor grid is 8 floor(H/8) x 8 floor(W/8), as the
// reference's SuperPoint on e.g. the ISEC cameras' 720x540 frames.
//
// Layout: activations NHWC bf16; 3x3 weights bf16 [Cout][3][3][Cin].  The 3x3 convs
// are implicit GEMMs on MFMA (k_conv3x3): a 16x16-pixel output tile per workgroup
// (8 waves, 2 image rows each), its 18x18 input halo staged once in LDS, the weights
// of one (tap, 64-channel) K-step double-buffered in LDS, D = W . P^T so each lane
// owns 4 consecutive output channels of one pixel; bias + ReLU (+ the following 2x2
// max-pool, across the wave's row pair and a lane-pair shuffle) fused in the epilogue.
// The 1x1 heads run on the GEMM kernels (gemm_bf16.hip); NMS, selection and
// descriptor sampling are small memory-bound kernels.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int TS = 16;          // output tile: TS x TS pixels
constexpr int HALO = TS + 2;    // 18
constexpr int KC = 64;          // channels per K-step

// ------------------------------------------------------------------ conv1a (Cin = 1)
// BGR uint8 -> cv2 gray (fixed point) / 255 -> 3x3 conv (f32) + bias + ReLU -> bf16 [.., 64]
__global__ __launch_bounds__(256) void k_sp_conv1a(const uint8_t* __restrict__ frames, long frame_stride, int H, int W,
                                                   int C, const float* __restrict__ w, const float* __restrict__ b,
                                                   bf16_t* __restrict__ out) {
    __shared__ float g[HALO][HALO];
    __shared__ float sw[64 * 9 + 64];
    const int bz = blockIdx.z;
    const int y0 = blockIdx.y * TS, x0 = blockIdx.x * TS;
    const uint8_t* img = frames + (size_t)bz * frame_stride;
    for (int i = threadIdx.x; i < 64 * 9; i += 256) sw[i] = w[i];
    if (threadIdx.x < 64) sw[576 + threadIdx.x] = b[threadIdx.x];
    for (int i = threadIdx.x; i < HALO * HALO; i += 256) {
        const int yy = y0 - 1 + i / HALO, xx = x0 - 1 + i % HALO;
        float v = 0.f;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const uint8_t* p = img + ((size_t)yy * W + xx) * C;
            int gy;
            if (C == 1) gy = p[0];
            else gy = (p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14;
            v = (float)gy / 255.0f;
        }
        g[i / HALO][i % HALO] = v;
    }
    __syncthreads();
    // thread -> 8 output channels (chunk t & 7) of one pixel per pass, 32 pixels per pass
    // in raster order of the tile: a wave-instruction stores 8 consecutive pixels' whole
    // 128-B channel vectors (1 KiB contiguous) instead of 16 B of 64 pixels
    const int ch = threadIdx.x & 7;
    float wr[8][9], br[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        br[j] = sw[576 + 8 * ch + j];
#pragma unroll
        for (int k = 0; k < 9; ++k) wr[j][k] = sw[(8 * ch + j) * 9 + k];
    }
#pragma unroll 2
    for (int pass = 0; pass < TS * TS / 32; ++pass) {
        const int p = pass * 32 + (threadIdx.x >> 3), ty = p / TS, tx = p % TS;
        const int y = y0 + ty, x = x0 + tx;
        if (y >= H || x >= W) continue;
        float nb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) nb[k] = g[ty + k / 3][tx + k % 3];
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                s0 += wr[j][k] * nb[k];
                s1 += wr[j + 1][k] * nb[k];
            }
            pk[j / 2] = pack_bf16x2(fmaxf(s0 + br[j], 0.f), fmaxf(s1 + br[j + 1], 0.f));
        }
        *reinterpret_cast<uint4*>(out + (((size_t)bz * H + y) * W + x) * 64 + 8 * ch) =
            make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
}

// ------------------------------------------------------------------ 3x3 conv, implicit GEMM
template <int CIN, int COUT_T, bool POOL>
__global__ __launch_bounds__(512) void k_conv3x3(const bf16_t* __restrict__ in, const bf16_t* __restrict__ wt,
                                                 const float* __restrict__ bias, bf16_t* __restrict__ out, int H,
                                                 int W, int Cout, int tiles_x) {
    // Row strides padded by 32 B (an odd multiple of 32 B in all): a ds_read_b128 lane group
    // ({0-3,12-15,20-27}, ... -- MI355X_MICROARCH.md LDS table) covers the 16 pixel columns
    // once with k-chunk a for 8 of them and a + 1 for the other 8; at 16-B chunk stride s
    // (mod 16) the slots (col * s + chunk) mod 16 are all distinct for s = 2 mod 4, while the
    // former +16 B padding (s odd) left 2-way bank conflicts on every halo and weight read
    // (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.44, profiles/r02p_pmc_lightglue.txt)
    constexpr int HS = CIN * 2 + 32;      // halo pixel stride (bytes)
    constexpr int BS = KC * 2 + 32;       // weight row stride (bytes)
    constexpr int NT = COUT_T / 16;       // N-tiles (output channels) per wave
    constexpr int STEPS = 9 * (CIN / KC);
    constexpr int HALO_BYTES = HALO * HALO * HS;
    static_assert(POOL || TS * TS * COUT_T * 2 <= HALO_BYTES + 2 * COUT_T * (KC * 2 + 16),
                  "output staging must fit in the (dead) halo + weight buffers");
    constexpr int B_BYTES = COUT_T * BS;
    __shared__ __attribute__((aligned(16))) char smem[HALO_BYTES + 2 * B_BYTES];
    char* sh = smem;
    char* sb = smem + HALO_BYTES;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bz = blockIdx.z, n0 = blockIdx.y * COUT_T;
    const int y0 = (blockIdx.x / tiles_x) * TS, x0 = (blockIdx.x % tiles_x) * TS;
    const bf16_t* img = in + (size_t)bz * H * W * CIN;

    // halo: 18 x 18 pixels x CIN channels, zero outside the image
    constexpr int CPP = CIN / 8;  // 16-B chunks per pixel
    for (int i = tid; i < HALO * HALO * CPP; i += 512) {
        const int px = i / CPP, ch = i % CPP;
        const int yy = y0 - 1 + px / HALO, xx = x0 - 1 + px % HALO;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
            v = *reinterpret_cast<const uint4*>(img + ((size_t)yy * W + xx) * CIN + ch * 8);
        *reinterpret_cast<uint4*>(sh + px * HS + ch * 16) = v;
    }
    // weights of one K-step: COUT_T rows x 64 channels (8 chunks per row)
    constexpr int WCH = COUT_T * 8;
    constexpr int WPT = (WCH + 511) / 512;
    // a vector type, not uint4: HIP struct copies are memcpys, which kept this array out of
    // registers (hipcc placed it in LDS, 16 KiB per workgroup, on the load path)
    typedef __attribute__((ext_vector_type(4))) unsigned int wvec;
    wvec wreg[WPT];
    auto wload = [&](int step) {
        const int tap = step / (CIN / KC), cc = step % (CIN / KC);
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int i = tid + j * 512;
            if (i < WCH) {
                const int r = i >> 3, ch = i & 7;
                wreg[j] = *reinterpret_cast<const wvec*>(wt + ((size_t)(n0 + r) * 9 + tap) * CIN + cc * KC + ch * 8);
            }
        }
    };
    auto wstore = [&](int buf) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int i = tid + j * 512;
            if (i < WCH) *reinterpret_cast<wvec*>(sb + buf * B_BYTES + (i >> 3) * BS + (i & 7) * 16) = wreg[j];
        }
    };
    wload(0);
    wstore(0);
    __syncthreads();

    f32x4 acc[2][NT];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int col = lane & 15, kg = lane >> 4;  // pixel column / k-group of this lane
    for (int step = 0; step < STEPS; ++step) {
        const int buf = step & 1;
        if (step + 1 < STEPS) wload(step + 1);
        const int tap = step / (CIN / KC), cc = step % (CIN / KC);
        const int dy = tap / 3, dx = tap % 3;
        const char* bb = sb + buf * B_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {  // two K = 32 halves of the 64-channel step
            const int choff = (cc * KC + kk * 32 + kg * 8) * 2;
            bf16x8 pf[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int hp = (2 * wave + r + dy) * HALO + col + dx;
                pf[r] = *reinterpret_cast<const bf16x8*>(sh + hp * HS + choff);
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const bf16x8 wf = *reinterpret_cast<const bf16x8*>(bb + (n * 16 + col) * BS + (kk * 32 + kg * 8) * 2);
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, pf[r], acc[r][n], 0, 0, 0);
            }
        }
        if (step + 1 < STEPS) wstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane holds channels n0 + n*16 + kg*4 .. +3 of pixel (row 2w + r, col)
    const int x = x0 + col;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int c = n0 + n * 16 + kg * 4;
        const float4 bv = *reinterpret_cast<const float4*>(bias + c);
        float v[2][4];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            v[r][0] = fmaxf(acc[r][n][0] + bv.x, 0.f);
            v[r][1] = fmaxf(acc[r][n][1] + bv.y, 0.f);
            v[r][2] = fmaxf(acc[r][n][2] + bv.z, 0.f);
            v[r][3] = fmaxf(acc[r][n][3] + bv.w, 0.f);
        }
        if (POOL) {
            float m[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // round first (the reference stores bf16 activations, then pools)
                const float a = bf16_to_f32(f32_to_bf16(v[0][j])), bq = bf16_to_f32(f32_to_bf16(v[1][j]));
                m[j] = fmaxf(a, bq);
                m[j] = fmaxf(m[j], __shfl_xor(m[j], 1, 64));
            }
            const int py = (y0 >> 1) + wave, px = x >> 1;
            if ((col & 1) == 0 && 2 * py + 1 < H && 2 * px + 1 < W) {
                uint2 o;
                o.x = pack_bf16x2(m[0], m[1]);
                o.y = pack_bf16x2(m[2], m[3]);
                *reinterpret_cast<uint2*>(out + (((size_t)bz * (H / 2) + py) * (W / 2) + px) * Cout + c) = o;
            }
        } else {  // stage the tile [256 px][COUT_T] (chunk c ^ (px & 7)) over the dead halo / weights
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int p = (2 * wave + r) * TS + col, cc = 2 * n + (kg >> 1);
                uint2 o;
                o.x = pack_bf16x2(v[r][0], v[r][1]);
                o.y = pack_bf16x2(v[r][2], v[r][3]);
                *reinterpret_cast<uint2*>(sh + p * (COUT_T * 2) + ((cc ^ (p & 7)) << 4) + 8 * (kg & 1)) = o;
            }
        }
    }
    if (!POOL) {  // each pixel's COUT_T channels as whole 16-B chunks: a wave-instruction
                  // stores 1 KiB of consecutive pixels' contiguous channel runs
        __syncthreads();
        constexpr int CPX = COUT_T / 8;  // 16-B chunks per pixel
#pragma unroll
        for (int it = 0; it < TS * TS * CPX / 512; ++it) {
            const int L = it * 512 + tid, p = L / CPX, cc = L % CPX;
            const int y = y0 + p / TS, xx = x0 + p % TS;
            if (y < H && xx < W)
                *reinterpret_cast<uint4*>(out + (((size_t)bz * H + y) * W + xx) * Cout + n0 + 8 * cc) =
                    *reinterpret_cast<const uint4*>(sh + p * (COUT_T * 2) + ((cc ^ (p & 7)) << 4));
        }
    }
}

// ------------------------------------------------------------------ detector head
// logits f32 [B*Hc*Wc, ld] (+ bias) -> softmax over 65 -> full-res scores [B, 8Hc, 8Wc]
__global__ void k_sp_scores(const float* __restrict__ logits, int ld, const float* __restrict__ bias, int B, int Hc,
                            int Wc, float* __restrict__ scores) {
    const long cell = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= (long)B * Hc * Wc) return;
    const float* l = logits + cell * ld;
    float v[65];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 65; ++c) {
        v[c] = l[c] + bias[c];
        mx = fmaxf(mx, v[c]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 65; ++c) {
        v[c] = expf(v[c] - mx);
        s += v[c];
    }
    const int b = (int)(cell / ((long)Hc * Wc)), rem = (int)(cell % ((long)Hc * Wc));
    const int cy = rem / Wc, cx = rem % Wc;
    const int H = Hc * 8, W = Wc * 8;
    float* o = scores + (size_t)b * H * W;
#pragma unroll
    for (int c = 0; c < 64; ++c) o[(size_t)(cy * 8 + c / 8) * W + cx * 8 + c % 8] = v[c] / s;
}

// ------------------------------------------------------------------ simple_nms
// separable (2r+1) max filter, -inf outside (max_pool2d padding semantics)
template <typename T>
__global__ void k_maxfilt(const T* __restrict__ in, T* __restrict__ out, int B, int H, int W, int r, int axis) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)B * H * W) return;
    const int x = (int)(i % W), y = (int)((i / W) % H);
    const T* base = in + (i - ((long)y * W + x));
    T m = in[i];
    if (axis == 0) {
        for (int d = -r; d <= r; ++d) {
            const int xx = x + d;
            if (xx >= 0 && xx < W) m = m > base[(long)y * W + xx] ? m : base[(long)y * W + xx];
        }
    } else {
        for (int d = -r; d <= r; ++d) {
            const int yy = y + d;
            if (yy >= 0 && yy < H) m = m > base[(long)yy * W + x] ? m : base[(long)yy * W + x];
        }
    }
    out[i] = m;
}

// mask = (s == maxpool(s))
__global__ void k_nms_init(const float* __restrict__ s, const float* __restrict__ mp, uint8_t* __restrict__ mask,
                           long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) mask[i] = s[i] == mp[i];
}
// supp = maxpool(mask) > 0 (given); ss = supp ? 0 : s
__global__ void k_nms_supp(const float* __restrict__ s, const uint8_t* __restrict__ supp, float* __restrict__ ss,
                           long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ss[i] = supp[i] ? 0.f : s[i];
}
// mask |= (ss == maxpool(ss)) & !supp
__global__ void k_nms_update(const float* __restrict__ ss, const float* __restrict__ mp,
                             const uint8_t* __restrict__ supp, uint8_t* __restrict__ mask, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) mask[i] = mask[i] | ((ss[i] == mp[i]) & !supp[i]);
}
// final: keep = mask ? s : 0; borders -> -1 (never above a positive threshold)
__global__ void k_nms_final(float* __restrict__ s, const uint8_t* __restrict__ mask, int B, int H, int W,
                            int border) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)B * H * W) return;
    const int x = (int)(i % W), y = (int)((i / W) % H);
    float v = mask[i] ? s[i] : 0.f;
    if (y < border || x < border || y >= H - border || x >= W - border) v = -1.f;
    s[i] = v;
}

// simple_nms(r = 4) + border + keep, fused: one workgroup per 32 x 64 output tile holds
// its scores with a 5 r halo (the dependency radius of the initial max-pool and two
// suppression rounds) in LDS and runs every max-pool (separable, -inf outside the image,
// as max_pool2d's padding) and mask update there -- one read of the score map (3.7x
// halo redundancy) and one write, instead of 16 full-resolution passes.  Out-of-place
// (neighbouring tiles read the input halo).
constexpr int NMS_TH = 32, NMS_TW = 64, NMS_HALO = 20;
constexpr int NMS_LH = NMS_TH + 2 * NMS_HALO, NMS_LW = NMS_TW + 2 * NMS_HALO, NMS_N = NMS_LH * NMS_LW;

template <typename T> struct Vec4;
template <> struct Vec4<float> { typedef float4 type; };
template <> struct Vec4<uint8_t> { typedef uchar4 type; };

template <typename T>
__device__ __forceinline__ T vmax_(T a, T b) { return a > b ? a : b; }
// floats: v_max_f32 / v_max3_f32 instead of a compare + select (+ its VCC wait states) per
// max -- the same values here: scores are finite or -inf, never NaN or -0
template <>
__device__ __forceinline__ float vmax_(float a, float b) { return fmaxf(a, b); }

// (2 R + 1) max filter of the tile, separable, R = 4: each thread produces 4 consecutive
// outputs from 12 inputs held in registers (one vector read per 4 in x, column reads in
// y).  Values outside the tile are -inf / 0 (never in a used output: see k_sp_nms).
// M (MLG_SP_NMS_MARGIN): only outputs at least M cells inside the tile border are
// produced -- pass k of the five needs margin 4 k (its input is valid 4 (k - 1) in, every
// later pass reads it only there), so the passes shrink instead of each covering the
// whole 72 x 104 region (47 % of the pooling work; the outputs at margin 20 unchanged).
#ifndef MLG_SP_NMS_MARGIN
#define MLG_SP_NMS_MARGIN 1
#endif
template <int M0, typename T>
__device__ __forceinline__ void nms_pool4(const T* in, T* tmp, T* out, T lo) {
    typedef typename Vec4<T>::type V;
    constexpr int M = MLG_SP_NMS_MARGIN ? M0 : 0;
    constexpr int GX = NMS_LW / 4, GY = NMS_LH / 4;
    constexpr int XR0 = M > 4 ? M - 4 : 0, XR1 = M > 4 ? NMS_LH - M + 4 : NMS_LH;  // x-pass rows
    constexpr int XG0 = M / 4, XGN = GX - 2 * (M / 4);                                // x-pass groups
    for (int i = threadIdx.x; i < (XR1 - XR0) * XGN; i += blockDim.x) {  // along x
        const int y = XR0 + i / XGN, g = XG0 + i % XGN;
        const V* row = reinterpret_cast<const V*>(in + y * NMS_LW);
        const V c = row[g];
        const V l = g > 0 ? row[g - 1] : V{lo, lo, lo, lo};
        const V r = g + 1 < GX ? row[g + 1] : V{lo, lo, lo, lo};
        const T v[12] = {l.x, l.y, l.z, l.w, c.x, c.y, c.z, c.w, r.x, r.y, r.z, r.w};
        T o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            T m = v[k];
#pragma unroll
            for (int d = 1; d <= 8; ++d) m = vmax_(m, v[k + d]);
            o[k] = m;
        }
        reinterpret_cast<V*>(tmp + y * NMS_LW)[g] = V{o[0], o[1], o[2], o[3]};
    }
    __syncthreads();
    constexpr int YG0 = M / 4, YGN = GY - 2 * (M / 4), YC0 = M, YCN = NMS_LW - 2 * M;  // y-pass
    for (int i = threadIdx.x; i < YGN * YCN; i += blockDim.x) {  // along y
        const int g = YG0 + i / YCN, x = YC0 + i % YCN, y0 = 4 * g;
        T v[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const int y = y0 - 4 + k;
            v[k] = (y >= 0 && y < NMS_LH) ? tmp[y * NMS_LW + x] : lo;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            T m = v[k];
#pragma unroll
            for (int d = 1; d <= 8; ++d) m = vmax_(m, v[k + d]);
            out[(y0 + k) * NMS_LW + x] = m;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(512) void k_sp_nms(const float* __restrict__ sc, float* __restrict__ out, int B, int H,
                                                int W, int border) {
    __shared__ __attribute__((aligned(16))) char nms_smem[(size_t)NMS_N * (4 * 4 + 3)];  // 142 KB: one per CU
    float* S = reinterpret_cast<float*>(nms_smem);
    float* A = S + NMS_N;
    float* Tm = A + NMS_N;
    float* P = Tm + NMS_N;
    uint8_t* MK = reinterpret_cast<uint8_t*>(P + NMS_N);
    uint8_t* SP = MK + NMS_N;
    uint8_t* TU = SP + NMS_N;
    const int tx = blockIdx.x, ty = blockIdx.y, b = blockIdx.z;
    const int ox = tx * NMS_TW - NMS_HALO, oy = ty * NMS_TH - NMS_HALO;
    const float* img = sc + (size_t)b * H * W;
    auto inside = [&](int i) {
        const int y = i / NMS_LW + oy, x = i % NMS_LW + ox;
        return y >= 0 && y < H && x >= 0 && x < W;
    };
    for (int i = threadIdx.x; i < NMS_N; i += blockDim.x) {
        const int y = i / NMS_LW + oy, x = i % NMS_LW + ox;
        S[i] = (y >= 0 && y < H && x >= 0 && x < W) ? img[(size_t)y * W + x] : -INFINITY;
    }
    __syncthreads();
    nms_pool4<4>(S, Tm, P, -INFINITY);  // max_mask = scores == max_pool(scores)
    for (int i = threadIdx.x; i < NMS_N; i += blockDim.x) MK[i] = inside(i) && S[i] == P[i];
    __syncthreads();
    auto iteration = [&](auto m) {  // margins 4 m + 4 (suppression), 4 m + 8 (new maxima)
        constexpr int MS = decltype(m)::value;
        nms_pool4<MS + 4>(MK, TU, SP, (uint8_t)0);  // supp_mask = max_pool(max_mask) > 0
        for (int i = threadIdx.x; i < NMS_N; i += blockDim.x) A[i] = inside(i) ? (SP[i] ? 0.f : S[i]) : -INFINITY;
        __syncthreads();
        nms_pool4<MS + 8>(A, Tm, P, -INFINITY);  // new_max_mask = supp_scores == max_pool(supp_scores)
        for (int i = threadIdx.x; i < NMS_N; i += blockDim.x)
            MK[i] = MK[i] | (inside(i) && A[i] == P[i] && !SP[i]);
        __syncthreads();
    };
    iteration(std::integral_constant<int, 4>{});
    iteration(std::integral_constant<int, 12>{});
    for (int i = threadIdx.x; i < NMS_TH * NMS_TW; i += blockDim.x) {
        const int ly = i / NMS_TW + NMS_HALO, lx = i % NMS_TW + NMS_HALO;
        const int y = ly + oy, x = lx + ox;
        if (y >= H || x >= W) continue;
        const int l = ly * NMS_LW + lx;
        float v = MK[l] ? S[l] : 0.f;
        if (y < border || x < border || y >= H - border || x >= W - border) v = -1.f;
        out[(size_t)b * H * W + (size_t)y * W + x] = v;
    }
}

// ------------------------------------------------------------------ selection
// One 1024-thread workgroup per frame.  Candidates (score > thr) are compacted in
// raster order; if there are more than k, the k-th largest score is found by a 4-pass
// radix select over the candidates, and the k selected (score desc, raster index asc)
// are bitonic-sorted in LDS.  Output keypoints are (x, y) floats.
constexpr int SEL_T = 1024;
constexpr int SEL_KMAX = 4096;
#ifndef MLG_SP_SEL_CHUNK
#define MLG_SP_SEL_CHUNK 1  // coalesced chunked candidate compaction (0: per-thread segments, A/B)
#endif

__global__ __launch_bounds__(SEL_T) void k_sp_select(const float* __restrict__ scores, int H, int W, float thr, int k,
                                                     uint32_t* __restrict__ cand_key, int32_t* __restrict__ cand_idx,
                                                     float* __restrict__ kpts, float* __restrict__ kscore,
                                                     int32_t* __restrict__ count) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const long HW = (long)H * W;
    const float* s = scores + b * HW;
    uint32_t* ck = cand_key + b * HW;
    int32_t* ci = cand_idx + b * HW;
    __shared__ int scan[SEL_T];
    __shared__ uint32_t hist[256];
    __shared__ unsigned long long keys[SEL_KMAX];
    __shared__ int sh_n, sh_gt;
    __shared__ uint32_t sh_prefix;

    // 1) ordered compaction of candidates
    if (MLG_SP_SEL_CHUNK) {
        // coalesced: chunks of SEL_T x 16 pixels, thread t holding pixels 16 t .. 16 t + 15
        // of the chunk (four float4 loads, a wave reads 4 KiB contiguous); raster-order
        // ranks from a wave shuffle scan of the per-thread counts plus the earlier waves'
        // totals (double-buffered, one barrier per chunk).  The same list, in the same
        // order, as the per-thread-segment form below (whose 300-pixel segments per lane
        // made every load touch 64 lines).
        __shared__ int wsum[2][SEL_T / 64];
        const int lane = tid & 63, wave = tid >> 6;
        constexpr int PER = 16, CH = SEL_T * PER;
        const bool vec = (HW & 3) == 0;
        int base = 0;
        for (long c0 = 0, it = 0; c0 < HW; c0 += CH, ++it) {
            const long p0 = c0 + (long)tid * PER;
            float v[PER];
#pragma unroll
            for (int q = 0; q < PER / 4; ++q) {
                const long i = p0 + 4 * q;
                if (vec && i + 3 < HW) {
                    const float4 f = *reinterpret_cast<const float4*>(s + i);
                    v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[4 * q + j] = i + j < HW ? s[i + j] : -INFINITY;
                }
            }
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < PER; ++j) cnt += v[j] > thr;
            int x = cnt;  // inclusive wave scan
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            if (lane == 63) wsum[it & 1][wave] = x;
            __syncthreads();
            int wbase = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < SEL_T / 64; ++w) {
                const int t = wsum[it & 1][w];
                wbase += w < wave ? t : 0;
                tot += t;
            }
            int off = base + wbase + x - cnt;
#pragma unroll
            for (int j = 0; j < PER; ++j)
                if (v[j] > thr) {
                    ck[off] = __float_as_uint(v[j]);
                    ci[off] = (int32_t)(p0 + j);
                    ++off;
                }
            base += tot;
        }
        if (tid == 0) sh_n = base;
        __syncthreads();
    } else {
        const long seg = (HW + SEL_T - 1) / SEL_T;
        const long a0 = tid * seg, a1 = min(HW, a0 + seg);
        int c = 0;
        for (long i = a0; i < a1; ++i) c += s[i] > thr;
        scan[tid] = c;
        __syncthreads();
        for (int o = 1; o < SEL_T; o <<= 1) {  // inclusive Hillis-Steele scan
            const int v = tid >= o ? scan[tid - o] : 0;
            __syncthreads();
            scan[tid] += v;
            __syncthreads();
        }
        int off = scan[tid] - c;
        for (long i = a0; i < a1; ++i) {
            const float v = s[i];
            if (v > thr) {
                ck[off] = __float_as_uint(v);
                ci[off] = (int32_t)i;
                ++off;
            }
        }
        if (tid == SEL_T - 1) sh_n = scan[SEL_T - 1];
        __syncthreads();
    }
    const int n = sh_n;
    float* kp = kpts + (size_t)b * k * 2;
    float* ks = kscore + (size_t)b * k;
    if (n <= k) {  // all of them, raster order
        for (int i = tid; i < n; i += SEL_T) {
            const int idx = ci[i];
            kp[2 * i] = (float)(idx % W);
            kp[2 * i + 1] = (float)(idx / W);
            ks[i] = __uint_as_float(ck[i]);
        }
        if (tid == 0) count[b] = n;
        return;
    }
    // 2) radix select of the k-th largest key (positive floats: bit order = value order)
    uint32_t prefix = 0, pmask = 0;
    int want = k;  // rank (1-based) of the key we look for among those matching the prefix
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < n; i += SEL_T) {
            const uint32_t key = ck[i];
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0, d = 255;
            for (; d > 0; --d) {
                if (acc + (int)hist[d] >= want) break;
                acc += hist[d];
            }
            sh_prefix = prefix | ((uint32_t)d << shift);
            sh_gt = acc;  // keys above digit d within the prefix
        }
        __syncthreads();
        want -= sh_gt;
        prefix = sh_prefix;
        pmask |= 255u << shift;
        __syncthreads();
    }
    const uint32_t T = prefix;  // the k-th largest key
    // count keys > T, then take (k - gt) keys == T in raster order
    if (tid == 0) sh_gt = 0;
    __syncthreads();
    int gt = 0;
    for (int i = tid; i < n; i += SEL_T) gt += ck[i] > T;
    atomicAdd(&sh_gt, gt);
    __syncthreads();
    const int need_eq = k - sh_gt;
    // ordered pass over equal keys (per-thread contiguous segments + scan)
    const int seg2 = (n + SEL_T - 1) / SEL_T;
    const int b0 = tid * seg2, b1 = min(n, b0 + seg2);
    int e = 0;
    for (int i = b0; i < b1; ++i) e += ck[i] == T;
    scan[tid] = e;
    __syncthreads();
    for (int o = 1; o < SEL_T; o <<= 1) {
        const int v = tid >= o ? scan[tid - o] : 0;
        __syncthreads();
        scan[tid] += v;
        __syncthreads();
    }
    // gather: keys > T anywhere, keys == T with rank < need_eq
    if (tid == 0) sh_n = 0;
    __syncthreads();
    int erank = scan[tid] - e;
    for (int i = b0; i < b1; ++i) {
        const uint32_t key = ck[i];
        bool take = key > T;
        if (key == T) {
            take = erank < need_eq;
            ++erank;
        }
        if (take) {
            const int slot = atomicAdd(&sh_n, 1);
            // sort key: score desc, raster index asc -> descending on (key, ~idx)
            keys[slot] = ((unsigned long long)key << 32) | (uint32_t)(~(uint32_t)ci[i]);
        }
    }
    __syncthreads();
    // 3) bitonic sort (descending) of k keys padded to a power of two
    int np2 = 1;
    while (np2 < k) np2 <<= 1;
    for (int i = k + tid; i < np2; i += SEL_T) keys[i] = 0ull;
    __syncthreads();
    for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < np2; i += SEL_T) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool desc = (i & size) == 0;
                    const unsigned long long a = keys[i], bq = keys[j];
                    if ((a < bq) == desc) { keys[i] = bq; keys[j] = a; }
                }
            }
            __syncthreads();
        }
    for (int i = tid; i < k; i += SEL_T) {
        const unsigned long long v = keys[i];
        const int idx = (int)(~(uint32_t)(v & 0xffffffffu));
        kp[2 * i] = (float)(idx % W);
        kp[2 * i + 1] = (float)(idx / W);
        ks[i] = __uint_as_float((uint32_t)(v >> 32));
    }
    if (tid == 0) count[b] = k;
}

// ------------------------------------------------------------------ descriptors
// One wave per keypoint: bilinear grid_sample (align_corners=True, zero padding) of the
// L2-normalised (convDb + bias) map at the keypoint, then L2-normalised.  4 channels
// per lane (256 = 64 x 4).
__device__ __forceinline__ float4 cell_normed(const float* __restrict__ d, const float* __restrict__ bias, int lane,
                                              bool valid) {
    if (!valid) return make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = *reinterpret_cast<const float4*>(d + lane * 4);
    const float4 bb = *reinterpret_cast<const float4*>(bias + lane * 4);
    v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
    const float n = sqrtf(wave_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w));
    const float inv = 1.0f / fmaxf(n, 1e-12f);
    return make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
}

__global__ __launch_bounds__(256) void k_sp_desc(const float* __restrict__ dmap, const float* __restrict__ bias, int B,
                                                 int Hc, int Wc, const float* __restrict__ kpts,
                                                 const int32_t* __restrict__ count, int k, float* __restrict__ desc,
                                                 uint16_t* __restrict__ desc_bf16) {
    const int lane = threadIdx.x & 63;
    const long gk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gk >= (long)B * k) return;
    const int b = (int)(gk / k), i = (int)(gk % k);
    float* out = desc + gk * 256;
    if (i >= count[b]) {
        *reinterpret_cast<float4*>(out + lane * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (desc_bf16) *reinterpret_cast<uint2*>(desc_bf16 + gk * 256 + lane * 4) = make_uint2(0, 0);
        return;
    }
    const float s = 8.0f;
    float kx = kpts[gk * 2], ky = kpts[gk * 2 + 1];
    kx = kx - s / 2 + 0.5f;
    ky = ky - s / 2 + 0.5f;
    kx = kx / ((float)Wc * s - s / 2 - 0.5f);
    ky = ky / ((float)Hc * s - s / 2 - 0.5f);
    kx = kx * 2.f - 1.f;
    ky = ky * 2.f - 1.f;
    const float ix = ((kx + 1.f) / 2.f) * (float)(Wc - 1);
    const float iy = ((ky + 1.f) / 2.f) * (float)(Hc - 1);
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
    const float wne = (ix - (float)x0) * ((float)y1 - iy);
    const float wsw = ((float)x1 - ix) * (iy - (float)y0);
    const float wse = (ix - (float)x0) * (iy - (float)y0);
    const float* base = dmap + (size_t)b * Hc * Wc * 256;
    auto in = [&](int x, int y) { return x >= 0 && x < Wc && y >= 0 && y < Hc; };
    auto at = [&](int x, int y) { return base + ((size_t)(in(x, y) ? y : 0) * Wc + (in(x, y) ? x : 0)) * 256; };
    const float4 vnw = cell_normed(at(x0, y0), bias, lane, in(x0, y0));
    const float4 vne = cell_normed(at(x1, y0), bias, lane, in(x1, y0));
    const float4 vsw = cell_normed(at(x0, y1), bias, lane, in(x0, y1));
    const float4 vse = cell_normed(at(x1, y1), bias, lane, in(x1, y1));
    float4 o;
    o.x = vnw.x * wnw + vne.x * wne + vsw.x * wsw + vse.x * wse;
    o.y = vnw.y * wnw + vne.y * wne + vsw.y * wsw + vse.y * wse;
    o.z = vnw.z * wnw + vne.z * wne + vsw.z * wsw + vse.z * wse;
    o.w = vnw.w * wnw + vne.w * wne + vsw.w * wsw + vse.w * wse;
    const float n = sqrtf(wave_sum(o.x * o.x + o.y * o.y + o.z * o.z + o.w * o.w));
    const float inv = 1.0f / fmaxf(n, 1e-12f);
    o.x *= inv; o.y *= inv; o.z *= inv; o.w *= inv;
    *reinterpret_cast<float4*>(out + lane * 4) = o;
    if (desc_bf16) {
        uint2 p;
        p.x = pack_bf16x2(o.x, o.y);
        p.y = pack_bf16x2(o.z, o.w);
        *reinterpret_cast<uint2*>(desc_bf16 + gk * 256 + lane * 4) = p;
    }
}

template <int CIN, int COUT_T, bool POOL>
int conv(const bf16_t* in, const bf16_t* w, const float* b, bf16_t* out, int B, int H, int W, int Cout,
         hipStream_t s) {
    if (Cout % COUT_T) return MLG_EINVAL;
    const int tx = (W + TS - 1) / TS, ty = (H + TS - 1) / TS;
    MlgProfScope prof(7, s, 2.0 * B * H * W * Cout * 9.0 * CIN);
    hipLaunchKernelGGL((k_conv3x3<CIN, COUT_T, POOL>), dim3(tx * ty, Cout / COUT_T, B), dim3(512), 0, s, in, w, b,
                       out, H, W, Cout, tx);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

#define SP_TRY(x)                   \
    do {                            \
        int rc_ = (x);              \
        if (rc_ != MLG_OK) return rc_; \
    } while (0)

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct SpLayout {
    size_t a, b, logits, dmap, scores, tmp, mask, supp, ckey, cidx, total;
};

SpLayout sp_layout(int B, int H, int W) {
    SpLayout L;
    const size_t HW = (size_t)H * W, cells = HW / 64;
    const size_t big = a256((size_t)B * HW * 64 * 2);  // conv1a output (largest activation)
    L.a = 0;
    L.b = L.a + big;
    L.logits = L.b + big;
    L.dmap = L.logits + a256((size_t)B * cells * 128 * 4);
    L.scores = L.dmap + a256((size_t)B * cells * 256 * 4);
    L.tmp = L.scores + a256((size_t)B * HW * 4);
    L.mask = L.tmp + a256((size_t)B * HW * 4 * 2);  // two f32 temporaries
    L.supp = L.mask + a256((size_t)B * HW);
    L.ckey = L.supp + a256((size_t)B * HW * 2);      // two u8 temporaries
    L.cidx = L.ckey + a256((size_t)B * HW * 4);
    L.total = L.cidx + a256((size_t)B * HW * 4);
    return L;
}

}  // namespace

size_t mlg_superpoint_ws_bytes(int B, int H, int W) {
    if (B <= 0 || H < 16 || W < 16) return 0;
    return sp_layout(B, H, W).total;
}

int mlg_superpoint_run(const mlg_sp_weights_i& w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                       float det_thr, int max_kp, int nms_radius, int border, void* ws, size_t ws_bytes, float* kpts,
                       float* kscores, float* desc, uint16_t* desc_bf16, int32_t* count, hipStream_t s) {
    if (B <= 0 || H < 16 || W < 16 || (C != 1 && C != 3 && C != 4) || max_kp <= 0 ||
        max_kp > SEL_KMAX || nms_radius < 0 || border < 0)
        return MLG_EINVAL;
    const SpLayout L = sp_layout(B, H, W);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* base = (char*)ws;
    bf16_t* A = (bf16_t*)(base + L.a);
    bf16_t* Bf = (bf16_t*)(base + L.b);
    float* logits = (float*)(base + L.logits);
    float* dmap = (float*)(base + L.dmap);
    float* sc = (float*)(base + L.scores);
    float* t0 = (float*)(base + L.tmp);
    float* t1 = t0 + (size_t)B * H * W;
    uint8_t* mask = (uint8_t*)(base + L.mask);
    uint8_t* u0 = (uint8_t*)(base + L.supp);
    uint8_t* u1 = u0 + (size_t)B * H * W;
    uint32_t* ckey = (uint32_t*)(base + L.ckey);
    int32_t* cidx = (int32_t*)(base + L.cidx);

    hipLaunchKernelGGL(k_sp_conv1a, dim3((W + TS - 1) / TS, (H + TS - 1) / TS, B), dim3(256), 0, s, frames,
                       frame_stride, H, W, C, w.conv1a_w, w.conv1a_b, A);
    MLG_LAUNCH_CHECK();
    int h = H, wd = W;
    SP_TRY((conv<64, 64, true>(A, w.w[0], w.b[0], Bf, B, h, wd, 64, s)));   // conv1b + pool
    h /= 2; wd /= 2;
    SP_TRY((conv<64, 64, false>(Bf, w.w[1], w.b[1], A, B, h, wd, 64, s)));  // conv2a
    SP_TRY((conv<64, 64, true>(A, w.w[2], w.b[2], Bf, B, h, wd, 64, s)));   // conv2b + pool
    h /= 2; wd /= 2;
    SP_TRY((conv<64, 128, false>(Bf, w.w[3], w.b[3], A, B, h, wd, 128, s)));   // conv3a
    SP_TRY((conv<128, 128, true>(A, w.w[4], w.b[4], Bf, B, h, wd, 128, s)));   // conv3b + pool
    h /= 2; wd /= 2;
    SP_TRY((conv<128, 128, false>(Bf, w.w[5], w.b[5], A, B, h, wd, 128, s)));  // conv4a
    SP_TRY((conv<128, 128, false>(A, w.w[6], w.b[6], Bf, B, h, wd, 128, s)));  // conv4b -> x (Bf)
    const int M = B * h * wd;
    bf16_t* cPa = A;
    bf16_t* cDa = A + (size_t)M * 256;
    SP_TRY((conv<128, 128, false>(Bf, w.w[7], w.b[7], cPa, B, h, wd, 256, s)));  // convPa
    SP_TRY((conv<128, 128, false>(Bf, w.w[9], w.b[9], cDa, B, h, wd, 256, s)));  // convDa
    SP_TRY(mlg_gemm_f32out(cPa, w.w[8], logits, M, 128, 256, s));                // convPb (65 of 128 rows)
    SP_TRY(mlg_gemm_f32out(cDa, w.w[10], dmap, M, 256, 256, s));                 // convDb
    hipLaunchKernelGGL(k_sp_scores, dim3((M + 255) / 256), dim3(256), 0, s, logits, 128, w.b[8], B, h, wd, sc);
    MLG_LAUNCH_CHECK();
    // the score map is 8 * floor(H / 8) x 8 * floor(W / 8): the encoder convolved the
    // full frame, its pools rounded down, and depth-to-space covers whole cells only
    H = 8 * h;
    W = 8 * wd;
    // simple_nms
    const float* nms_out = sc;
    if (nms_radius == 4) {  // fused (SuperPoint's default radius)
        hipLaunchKernelGGL(k_sp_nms, dim3((unsigned)((W + NMS_TW - 1) / NMS_TW), (unsigned)((H + NMS_TH - 1) / NMS_TH),
                                          (unsigned)B),
                           dim3(512), 0, s, sc, t0, B, H, W, border);
        MLG_LAUNCH_CHECK();
        nms_out = t0;
    } else {  // multi-pass at full resolution
        const long n = (long)B * H * W;
        const dim3 g((unsigned)((n + 255) / 256)), t(256);
        auto maxpool_f = [&](const float* in, float* out) {
            hipLaunchKernelGGL(k_maxfilt<float>, g, t, 0, s, in, t1, B, H, W, nms_radius, 0);
            hipLaunchKernelGGL(k_maxfilt<float>, g, t, 0, s, (const float*)t1, out, B, H, W, nms_radius, 1);
        };
        maxpool_f(sc, t0);
        hipLaunchKernelGGL(k_nms_init, g, t, 0, s, sc, t0, mask, n);
        for (int it = 0; it < 2; ++it) {
            hipLaunchKernelGGL(k_maxfilt<uint8_t>, g, t, 0, s, mask, u1, B, H, W, nms_radius, 0);
            hipLaunchKernelGGL(k_maxfilt<uint8_t>, g, t, 0, s, (const uint8_t*)u1, u0, B, H, W, nms_radius, 1);
            hipLaunchKernelGGL(k_nms_supp, g, t, 0, s, sc, u0, t0, n);   // t0 = supp_scores
            hipLaunchKernelGGL(k_maxfilt<float>, g, t, 0, s, (const float*)t0, t1, B, H, W, nms_radius, 0);
            float* mp = (float*)ckey;  // scratch (candidates are written later)
            hipLaunchKernelGGL(k_maxfilt<float>, g, t, 0, s, (const float*)t1, mp, B, H, W, nms_radius, 1);
            hipLaunchKernelGGL(k_nms_update, g, t, 0, s, t0, mp, u0, mask, n);
        }
        hipLaunchKernelGGL(k_nms_final, g, t, 0, s, sc, mask, B, H, W, border);
        MLG_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_sp_select, dim3(B), dim3(SEL_T), 0, s, nms_out, H, W, det_thr, max_kp, ckey, cidx, kpts, kscores,
                       count);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sp_desc, dim3((unsigned)(((long)B * max_kp + 3) / 4)), dim3(256), 0, s, dmap, w.b[10], B, h,
                       wd, kpts, count, max_kp, desc, desc_bf16);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
