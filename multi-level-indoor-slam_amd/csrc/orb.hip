// ORB + brute-force Hamming matcher: the reference's fallback matcher
// (LightGlue._load_fallback / _detect_and_match_fallback,
// scripts/semantic_gating/geometric_verification.py:244-248, 314-350:
// cv2.ORB_create(nfeatures=max_keypoints).detectAndCompute on BGR2GRAY frames,
// cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match, sorted by distance).
//
// Restated from OpenCV's ORB (orb.cpp) -- the algorithm and its deviations are listed in
// oracle/csrc/orb.c, which this file matches bit for bit.  MI355X shape:
//   * a batch of F frames at once; every pixel stage is one launch per pyramid level
//     over all frames (gray, INTER_LINEAR_EXACT pyramid, FAST-9 score map, 3x3 NMS + border
//     + per-(frame, level) candidate lists and FAST-score histograms, 7x7 Gaussian);
//   * retainBest twice without a global sort: the FAST-score threshold of the 2n best
//     comes from the 256-bin histogram (ties at it kept, as retainBest keeps them), the
//     Harris responses of the survivors are sorted in LDS by one workgroup per
//     (frame, level) with a bitonic network on 64-bit (response, y, x) keys;
//   * orientation (intensity centroid + fastAtan2) and rBRIEF per keypoint;
//   * matching: one thread per query descriptor against the train set streamed through
//     LDS (4 x 64-bit popcounts per pair), both directions, then cross-check and a
//     stable counting sort by distance per pair in one workgroup.
#include <stdint.h>

#include "common.h"
#include "kernels.h"
#include "../../include/mlgate.h"

namespace {

constexpr int NL = MLG_ORB_LEVELS;
constexpr int SORT_CAP = 8192;  // survivors of the FAST retainBest per (frame, level)

struct OrbGeom {
    int H, W, F, nfeat_total, max_kp;
    int lw[NL], lh[NL], nfeat[NL];
    long loff[NL];   // byte offset of level l inside one frame's pyramid image
    long lcap[NL];   // candidate capacity of level l
    long coff[NL];   // candidate-list offset of level l inside one frame's lists
    float lscale[NL];
    long pyr_bytes;  // per frame
    long cand_per_frame;
    int fast_t, edge;
    int umax[16];
    float gk[7];
};


__global__ void k_orb_gray(const uint8_t* __restrict__ frames, long stride, int C, OrbGeom g,
                           uint8_t* __restrict__ pyr) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long px = (long)g.H * g.W;
    if (e >= px * g.F) return;
    const int f = (int)(e / px);
    const long i = e - (long)f * px;
    const uint8_t* p = frames + f * stride + i * C;
    pyr[(long)f * g.pyr_bytes + i] =
        (uint8_t)(C >= 3 ? (p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14 : p[0]);
}

// cv::resize(..., INTER_LINEAR_EXACT) of level l - 1 into level l (OpenCV resize.cpp
// resize_bitExact on 8U; oracle/csrc/orb.c resize_linear_exact_u8): binary64 source
// coordinate, 8-bit tap weights, 16-bit horizontal sums, (h0 c0 + h1 c1 + 2^15) >> 16.
__device__ __forceinline__ void exact_tap(int d, int dsize, int ssize, int& i0, uint32_t& c1) {
    const double inv = __ddiv_rn((double)dsize, (double)ssize), scale = __ddiv_rn(1.0, inv);
    const double f = __dsub_rn(__dmul_rn(scale, __dadd_rn((double)d, 0.5)), 0.5);
    const int i = (int)floor(f);
    if (i < 0 || ssize <= 1) {
        i0 = 0;
        c1 = 0;
    } else if (i >= ssize - 1) {
        i0 = ssize - 1;
        c1 = 0;
    } else {
        i0 = i;
        c1 = (uint32_t)__double2int_rn(__dmul_rn(__dsub_rn(f, (double)i), 256.0));
    }
}

__global__ void k_orb_resize(OrbGeom g, int l, uint8_t* __restrict__ pyr) {
    const int W = g.lw[l - 1], H = g.lh[l - 1], DW = g.lw[l], DH = g.lh[l];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)g.F * DH * DW) return;
    const int dx = (int)(e % DW), dy = (int)((e / DW) % DH), f = (int)(e / ((long)DW * DH));
    int x0, y0;
    uint32_t cx1, cy1;
    exact_tap(dx, DW, W, x0, cx1);
    exact_tap(dy, DH, H, y0, cy1);
    const int x1 = x0 + 1 < W ? x0 + 1 : x0, y1 = y0 + 1 < H ? y0 + 1 : y0;
    const uint32_t cx0 = 256u - cx1, cy0 = 256u - cy1;
    const uint8_t* src = pyr + (long)f * g.pyr_bytes + g.loff[l - 1];
    const uint8_t* r0 = src + (long)y0 * W;
    const uint8_t* r1 = src + (long)y1 * W;
    const uint32_t h0 = cx0 * r0[x0] + cx1 * r0[x1], h1 = cx0 * r1[x0] + cx1 * r1[x1];
    pyr[(long)f * g.pyr_bytes + g.loff[l] + e % ((long)DW * DH)] = (uint8_t)((h0 * cy0 + h1 * cy1 + 32768u) >> 16);
}

__constant__ int8_t CIRC[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                   {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// FAST-9 score map (OpenCV cornerScore<16>: the largest threshold at which the pixel is
// still a corner, 0 = no corner) for 3 <= x < w - 3, 3 <= y < h - 3; 0 elsewhere.
__global__ void k_orb_fast(OrbGeom g, int l, const uint8_t* __restrict__ pyr, uint8_t* __restrict__ score) {
    const int w = g.lw[l], h = g.lh[l];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)g.F * w * h) return;
    const int x = (int)(e % w), y = (int)((e / w) % h), f = (int)(e / ((long)w * h));
    const long base = (long)f * g.pyr_bytes + g.loff[l];
    int s = 0;
    if (x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
        const uint8_t* img = pyr + base;
        const int v = img[y * w + x];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = img[(y + CIRC[k][1]) * w + x + CIRC[k][0]] - v;
        int bb = -1, bd = -1;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            int mb = d[k], md = -d[k];
#pragma unroll
            for (int j = 1; j < 9; ++j) {
                mb = min(mb, d[(k + j) & 15]);
                md = min(md, -d[(k + j) & 15]);
            }
            bb = max(bb, mb);
            bd = max(bd, md);
        }
        const int m = max(bb, bd);
        s = m > g.fast_t ? m - 1 : 0;
    }
    score[base + (long)y * w + x] = (uint8_t)s;
}

// Strict 3x3 maxima inside the edge border -> candidate list + FAST-score histogram of
// (frame, level).  List order is arbitrary (atomics); everything after is order-free.
__global__ void k_orb_nms(OrbGeom g, int l, const uint8_t* __restrict__ score, uint32_t* __restrict__ cand,
                          int* __restrict__ ccount, int* __restrict__ hist) {
    const int w = g.lw[l], h = g.lh[l], E = g.edge;
    const int iw = w - 2 * E, ih = h - 2 * E;
    if (iw <= 0 || ih <= 0) return;
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)g.F * iw * ih) return;
    const int x = E + (int)(e % iw), y = E + (int)((e / iw) % ih), f = (int)(e / ((long)iw * ih));
    const uint8_t* sc = score + (long)f * g.pyr_bytes + g.loff[l];
    const int s = sc[y * w + x];
    if (!s) return;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx)
            if ((dx || dy) && sc[(y + dy) * w + x + dx] >= s) return;
    const int seg = f * NL + l;
    const int slot = atomicAdd(ccount + seg, 1);
    if (slot < g.lcap[l]) cand[(long)f * g.cand_per_frame + g.coff[l] + slot] = ((uint32_t)s << 24) | (uint32_t)(y * w + x);
    atomicAdd(hist + seg * 256 + s, 1);
}

__device__ __forceinline__ int reflect101(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) as OpenCV runs it on ORB's pyramid
// submatrices: sepFilter2D with the float kernel -- row pass k0 x0 + ... + k6 x6 left to
// right, symmetric column pass k3 c + k4 (u1 + d1) + k5 (u2 + d2) + k6 (u3 + d3), round
// half to even, saturate (every operation rounded separately, as oracle/csrc/orb.c).
__device__ __forceinline__ float blur_row(const uint8_t* row, const int* xs, const float* k) {
    float s = __fmul_rn(k[0], (float)row[xs[0]]);
#pragma unroll
    for (int t = 1; t < 7; ++t) s = __fadd_rn(s, __fmul_rn(k[t], (float)row[xs[t]]));
    return s;
}

__global__ void k_orb_blur(OrbGeom g, int l, const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur) {
    const int w = g.lw[l], h = g.lh[l];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)g.F * w * h) return;
    const int x = (int)(e % w), y = (int)((e / w) % h), f = (int)(e / ((long)w * h));
    const long base = (long)f * g.pyr_bytes + g.loff[l];
    const uint8_t* img = pyr + base;
    int xs[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) xs[k] = reflect101(x + k - 3, w);
    float s = __fmul_rn(g.gk[3], blur_row(img + (long)y * w, xs, g.gk));
#pragma unroll
    for (int t = 1; t <= 3; ++t) {
        const float up = blur_row(img + (long)reflect101(y - t, h) * w, xs, g.gk);
        const float dn = blur_row(img + (long)reflect101(y + t, h) * w, xs, g.gk);
        s = __fadd_rn(s, __fmul_rn(g.gk[3 + t], __fadd_rn(dn, up)));
    }
    const int v = __float2int_rn(s);
    blur[base + (long)y * w + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__device__ __forceinline__ float harris_resp(const uint8_t* img, int W, int x, int y) {
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const uint8_t* p = img + (y - 3 + i) * W + (x - 3 + j);
            const int ix = (p[1] - p[-1]) * 2 + (p[-W + 1] - p[-W - 1]) + (p[W + 1] - p[W - 1]);
            const int iy = (p[W] - p[-W]) * 2 + (p[W - 1] - p[-W - 1]) + (p[W + 1] - p[-W + 1]);
            a += ix * ix;
            b += iy * iy;
            c += ix * iy;
        }
    const float scale = 1.f / ((1 << 2) * 7 * 255.f);
    const float s4 = __fmul_rn(__fmul_rn(__fmul_rn(scale, scale), scale), scale);
    const float A = (float)a, B = (float)b, C = (float)c;
    const float t = __fadd_rn(A, B);
    return __fmul_rn(__fsub_rn(__fsub_rn(__fmul_rn(A, B), __fmul_rn(C, C)), __fmul_rn(__fmul_rn(0.04f, t), t)), s4);
}

// (response desc, y asc, x asc) as one ascending 64-bit key
__device__ __forceinline__ uint64_t sort_key(float r, int y, int x) {
    uint32_t u = __float_as_uint(r);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending float order
    return ((uint64_t)(~u) << 32) | ((uint32_t)y << 16) | (uint32_t)x;
}

// One workgroup per (frame, level): retainBest(2 n) by FAST score, Harris, retainBest(n)
// by Harris; survivors (x, y, response) in key order into the level's output slots.
__global__ __launch_bounds__(256) void k_orb_select(OrbGeom g, const uint8_t* __restrict__ pyr,
                                                    const uint32_t* __restrict__ cand,
                                                    const int* __restrict__ ccount, const int* __restrict__ hist,
                                                    int4* __restrict__ sel, int* __restrict__ scount) {
    __shared__ uint64_t keys[SORT_CAP];
    __shared__ int s_thr, s_n;
    const int seg = blockIdx.x, f = seg / NL, l = seg % NL, tid = threadIdx.x;
    const int w = g.lw[l];
    const int total = min(ccount[seg], (int)g.lcap[l]);
    const int n1 = 2 * g.nfeat[l], n2 = g.nfeat[l];
    if (tid == 0) {
        int thr = 0;
        if (ccount[seg] > g.lcap[l]) {
            thr = -1;  // list overflow: reported below
        } else if (total > n1) {
            int acc = 0;
            for (int s = 255; s > 0; --s) {
                acc += hist[seg * 256 + s];
                if (acc >= n1) { thr = s; break; }
            }
        }
        s_thr = thr;
        s_n = 0;
    }
    __syncthreads();
    const int thr = s_thr;
    if (thr < 0 || n2 <= 0) {
        if (tid == 0) scount[seg] = thr < 0 ? -1 : 0;
        return;
    }
    const uint8_t* img = pyr + (long)f * g.pyr_bytes + g.loff[l];
    const uint32_t* cl = cand + (long)f * g.cand_per_frame + g.coff[l];
    // candidate word: FAST score << 24 | pixel index
    for (int i = tid; i < total; i += 256) {
        const uint32_t c = cl[i];
        if ((int)(c >> 24) < thr) continue;
        const int pix = (int)(c & 0xffffffu), y = pix / w, x = pix - y * w;
        const int slot = atomicAdd(&s_n, 1);
        if (slot < SORT_CAP) keys[slot] = sort_key(harris_resp(img, w, x, y), y, x);
    }
    __syncthreads();
    const int K = s_n;
    if (K > SORT_CAP) {
        if (tid == 0) scount[seg] = -2;
        return;
    }
    int P = 1;
    while (P < K) P <<= 1;
    for (int i = K + tid; i < P; i += 256) keys[i] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = keys[i], b = keys[ixj];
                    if (((i & k) == 0) == (a > b)) { keys[i] = b; keys[ixj] = a; }
                }
            }
            __syncthreads();
        }
    // retainBest(n): all keys whose response equals or beats the n-th
    int fin = K;
    if (K > n2) {
        const uint32_t hi = (uint32_t)(keys[n2 - 1] >> 32);
        fin = n2;
        while (fin < K && (uint32_t)(keys[fin] >> 32) == hi) ++fin;  // same response (ties)
    }
    const int cap = (int)(g.lcap[l]);
    for (int i = tid; i < fin && i < cap; i += 256) {
        const uint64_t kk = keys[i];
        uint32_t u = ~(uint32_t)(kk >> 32);
        u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
        sel[(long)f * g.cand_per_frame + g.coff[l] + i] =
            make_int4((int)(kk & 0xffffu), (int)((kk >> 16) & 0xffffu), (int)u, l);
    }
    if (tid == 0) scount[seg] = fin;
}

// Per frame: concatenate the levels' survivors (level order) into the output slots.
__global__ void k_orb_gather(OrbGeom g, const int* __restrict__ scount, int* __restrict__ kstart,
                             int32_t* __restrict__ count) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= g.F) return;
    int acc = 0, bad = 0;
    for (int l = 0; l < NL; ++l) {
        const int c = scount[f * NL + l];
        kstart[f * NL + l] = acc;
        if (c < 0) bad = c;
        else acc += c;
    }
    count[f] = bad ? bad : min(acc, g.max_kp);
}

__device__ float fast_atan2_deg(float y, float x) {
    const float k = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = __fmul_rn(0.9997878412794807f, k), p3 = __fmul_rn(-0.3258083974640975f, k);
    const float p5 = __fmul_rn(0.1555786518463281f, k), p7 = __fmul_rn(-0.04432655554792128f, k);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, (float)2.220446049250313e-16));
        c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, (float)2.220446049250313e-16));
        c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f,
                      __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// One thread per output keypoint: intensity-centroid angle on the level image, rBRIEF
// on the blurred level, level-0 coordinates.
__global__ void k_orb_describe(OrbGeom g, const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                               const int4* __restrict__ sel, const int* __restrict__ scount,
                               const int* __restrict__ kstart, const int32_t* __restrict__ count,
                               const int16_t* __restrict__ pattern, float* __restrict__ kpts, float* __restrict__ resp,
                               float* __restrict__ angle, int32_t* __restrict__ level, uint8_t* __restrict__ desc) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int f = (int)(e / g.max_kp), k = (int)(e % g.max_kp);
    if (f >= g.F || k >= count[f]) return;
    int l = 0;
    while (l + 1 < NL && kstart[f * NL + l + 1] <= k) ++l;
    const int4 s = sel[(long)f * g.cand_per_frame + g.coff[l] + (k - kstart[f * NL + l])];
    const int x = s.x, y = s.y, w = g.lw[l];
    const uint8_t* img = pyr + (long)f * g.pyr_bytes + g.loff[l];
    const uint8_t* center = img + (long)y * w + x;
    int m01 = 0, m10 = 0;
    for (int u = -15; u <= 15; ++u) m10 += u * center[u];
    for (int v = 1; v <= 15; ++v) {
        int vsum = 0;
        const int d = g.umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = center[u + v * w], vm = center[u - v * w];
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    const float ang = fast_atan2_deg((float)m01, (float)m10);
    const long o = (long)f * g.max_kp + k;
    kpts[2 * o] = __fmul_rn((float)x, g.lscale[l]);
    kpts[2 * o + 1] = __fmul_rn((float)y, g.lscale[l]);
    resp[o] = __int_as_float(s.z);
    angle[o] = ang;
    level[o] = l;
    const float rad = __fmul_rn(ang, (float)(3.1415926535897932384626433832795 / 180.f));
    const float a = (float)cos((double)rad), b = (float)sin((double)rad);
    const uint8_t* bc = blur + (long)f * g.pyr_bytes + g.loff[l] + (long)y * w + x;
    uint32_t words[8];
#pragma unroll
    for (int wd = 0; wd < 8; ++wd) {
        uint32_t word = 0;
#pragma unroll
        for (int bit = 0; bit < 32; ++bit) {
            const int pi = wd * 32 + bit;
            const float x0 = pattern[4 * pi], y0 = pattern[4 * pi + 1];
            const float x1 = pattern[4 * pi + 2], y1 = pattern[4 * pi + 3];
            const int r0 = __float2int_rn(__fadd_rn(__fmul_rn(x0, b), __fmul_rn(y0, a)));
            const int c0 = __float2int_rn(__fsub_rn(__fmul_rn(x0, a), __fmul_rn(y0, b)));
            const int r1 = __float2int_rn(__fadd_rn(__fmul_rn(x1, b), __fmul_rn(y1, a)));
            const int c1 = __float2int_rn(__fsub_rn(__fmul_rn(x1, a), __fmul_rn(y1, b)));
            word |= (uint32_t)(bc[r0 * w + c0] < bc[r1 * w + c1]) << bit;
        }
        words[wd] = word;
    }
    uint4* dst = reinterpret_cast<uint4*>(desc + o * 32);
    dst[0] = make_uint4(words[0], words[1], words[2], words[3]);
    dst[1] = make_uint4(words[4], words[5], words[6], words[7]);
}

// Nearest neighbour by Hamming distance (first minimum) of every query descriptor of a
// pair in the train set; dir 0: a -> b, dir 1: b -> a.
__global__ __launch_bounds__(256) void k_orb_nn(const uint8_t* __restrict__ desc, const int32_t* __restrict__ count,
                                                int max_kp, const int32_t* __restrict__ pa,
                                                const int32_t* __restrict__ pb, int dir, int* __restrict__ best,
                                                int* __restrict__ bdist) {
    __shared__ ulonglong4 tr[256];
    const int p = blockIdx.y, q = blockIdx.x * 256 + threadIdx.x;
    const int fq = dir ? pb[p] : pa[p], ft = dir ? pa[p] : pb[p];
    const int nq = count[fq], nt = count[ft];
    if (blockIdx.x * 256 >= nq) return;
    ulonglong4 qd = make_ulonglong4(0, 0, 0, 0);
    if (q < nq) qd = *reinterpret_cast<const ulonglong4*>(desc + ((long)fq * max_kp + q) * 32);
    int bi = -1, bd = 1 << 30;
    for (int t0 = 0; t0 < nt; t0 += 256) {
        __syncthreads();
        if (t0 + (int)threadIdx.x < nt)
            tr[threadIdx.x] = *reinterpret_cast<const ulonglong4*>(desc + ((long)ft * max_kp + t0 + threadIdx.x) * 32);
        __syncthreads();
        const int m = min(256, nt - t0);
        for (int j = 0; j < m; ++j) {
            const ulonglong4 t = tr[j];
            const int d = __popcll(qd.x ^ t.x) + __popcll(qd.y ^ t.y) + __popcll(qd.z ^ t.z) + __popcll(qd.w ^ t.w);
            if (d < bd) { bd = d; bi = t0 + j; }
        }
    }
    if (q < nq) {
        best[((long)dir * gridDim.y + p) * max_kp + q] = bi;
        bdist[((long)dir * gridDim.y + p) * max_kp + q] = bd;
    }
}

// Cross-check and stable counting sort by distance: one workgroup per pair.
__global__ __launch_bounds__(256) void k_orb_cross(const int32_t* __restrict__ count, int max_kp,
                                                   const int32_t* __restrict__ pa, int P, const int* __restrict__ best,
                                                   const int* __restrict__ bdist, int32_t* __restrict__ oq,
                                                   int32_t* __restrict__ ot, int32_t* __restrict__ od,
                                                   int32_t* __restrict__ nmatch) {
    __shared__ int hist[257], base[257];
    __shared__ int dch[256];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nq = count[pa[p]];
    const int* b12 = best + (long)p * max_kp;
    const int* d12 = bdist + (long)p * max_kp;
    const int* b21 = best + ((long)P + p) * max_kp;
    for (int i = tid; i < 257; i += 256) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < nq; i += 256) {
        const int j = b12[i];
        if (j >= 0 && b21[j] == i) atomicAdd(&hist[d12[i]], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int d = 0; d < 257; ++d) { base[d] = acc; acc += hist[d]; }
        nmatch[p] = acc;
    }
    __syncthreads();
    for (int c0 = 0; c0 < nq; c0 += 256) {
        const int i = c0 + tid;
        int d = -1;
        if (i < nq) {
            const int j = b12[i];
            if (j >= 0 && b21[j] == i) d = d12[i];
        }
        dch[tid] = d;
        __syncthreads();
        if (d >= 0) {
            int r = 0;
            for (int t = 0; t < tid; ++t) r += dch[t] == d;
            const long o = (long)p * max_kp + base[d] + r;
            oq[o] = i;
            ot[o] = b12[i];
            od[o] = d;
        }
        __syncthreads();
        if (tid == 0)
            for (int t = 0; t < 256; ++t)
                if (dch[t] >= 0) ++base[dch[t]];
        __syncthreads();
    }
}

long a256(long x) { return (x + 255) & ~255L; }

struct OrbLayout {
    long pyr, blur, score, cand, sel, ccount, hist, scount, kstart, total;
};

OrbLayout orb_layout(const OrbGeom& g) {
    OrbLayout L{};
    long o = 0;
    L.pyr = o;    o += a256(g.pyr_bytes * g.F);
    L.blur = o;   o += a256(g.pyr_bytes * g.F);
    L.score = o;  o += a256(g.pyr_bytes * g.F);
    L.cand = o;   o += a256(g.cand_per_frame * g.F * 4);
    L.sel = o;    o += a256(g.cand_per_frame * g.F * 16);
    L.ccount = o; o += a256((long)g.F * NL * 4);
    L.hist = o;   o += a256((long)g.F * NL * 256 * 4);
    L.scount = o; o += a256((long)g.F * NL * 4);
    L.kstart = o; o += a256((long)g.F * NL * 4);
    L.total = o;
    return L;
}

bool make_geom(const mlg_orb_params* p, int F, int H, int W, int max_kp, OrbGeom& g) {
    if (!mlg_head_ok(p, MLG_ABI_VERSION) || F <= 0 || H < 16 || W < 16 || max_kp <= 0 || H > 65535 || W > 65535) return false;
    g = OrbGeom{};
    g.H = H; g.W = W; g.F = F; g.max_kp = max_kp;
    g.fast_t = p->fast_threshold;
    g.edge = p->edge_threshold;
    long off = 0, coff = 0;
    for (int l = 0; l < NL; ++l) {
        g.lw[l] = p->level_w[l];
        g.lh[l] = p->level_h[l];
        g.nfeat[l] = p->level_features[l];
        g.lscale[l] = p->level_scale[l];
        if (g.lw[l] < 1 || g.lh[l] < 1 || g.nfeat[l] < 0) return false;
        g.loff[l] = off;
        off += ((long)g.lw[l] * g.lh[l] + 15) & ~15L;
        const long iw = std::max(0, g.lw[l] - 2 * g.edge), ih = std::max(0, g.lh[l] - 2 * g.edge);
        g.lcap[l] = ((iw + 1) / 2) * ((ih + 1) / 2) + 16;  // strict 3x3 maxima: <= 1 per 2x2 cell
        g.coff[l] = coff;
        coff += (g.lcap[l] + 3) & ~3L;
    }
    if (g.lw[0] != W || g.lh[0] != H || (long)W * H >= (1L << 24)) return false;
    g.pyr_bytes = (off + 255) & ~255L;
    g.cand_per_frame = coff;
    for (int i = 0; i < 16; ++i) g.umax[i] = p->umax[i];
    for (int i = 0; i < 7; ++i) g.gk[i] = p->gauss[i];
    return true;
}

inline unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" {

size_t mlg_orb_workspace_bytes(const mlg_orb_params* p, int F, int H, int W, int max_kp) {
    OrbGeom g;
    if (!make_geom(p, F, H, W, max_kp, g)) return 0;
    return (size_t)orb_layout(g).total;
}

int mlg_orb_detect(const mlg_orb_params* p, const int16_t* pattern, const uint8_t* frames, long frame_stride, int F,
                   int H, int W, int C, int max_kp, void* ws, size_t ws_bytes, float* keypoints, float* responses,
                   float* angles, int32_t* levels, uint8_t* descriptors, int32_t* counts, void* stream) {
    OrbGeom g;
    if (!make_geom(p, F, H, W, max_kp, g) || !pattern || !frames || (C != 1 && C != 3 && C != 4) ||
        frame_stride < (long)H * W * C)
        return MLG_EINVAL;
    const OrbLayout L = orb_layout(g);
    if (!ws || ws_bytes < (size_t)L.total) return MLG_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    char* b = (char*)ws;
    uint8_t* pyr = (uint8_t*)(b + L.pyr);
    uint8_t* blur = (uint8_t*)(b + L.blur);
    uint8_t* score = (uint8_t*)(b + L.score);
    uint32_t* cand = (uint32_t*)(b + L.cand);
    int4* sel = (int4*)(b + L.sel);
    int* ccount = (int*)(b + L.ccount);
    int* hist = (int*)(b + L.hist);
    int* scount = (int*)(b + L.scount);
    int* kstart = (int*)(b + L.kstart);
    if (hipMemsetAsync(ccount, 0, sizeof(int) * F * NL, s) != hipSuccess ||
        hipMemsetAsync(hist, 0, sizeof(int) * F * NL * 256, s) != hipSuccess)
        return MLG_EHIP;
    hipLaunchKernelGGL(k_orb_gray, dim3(blocks((long)F * H * W)), dim3(256), 0, s, frames, frame_stride, C, g, pyr);
    MLG_LAUNCH_CHECK();
    for (int l = 1; l < NL; ++l) {
        hipLaunchKernelGGL(k_orb_resize, dim3(blocks((long)F * g.lw[l] * g.lh[l])), dim3(256), 0, s, g, l, pyr);
        MLG_LAUNCH_CHECK();
    }
    for (int l = 0; l < NL; ++l) {
        const long px = (long)F * g.lw[l] * g.lh[l];
        hipLaunchKernelGGL(k_orb_fast, dim3(blocks(px)), dim3(256), 0, s, g, l, pyr, score);
        MLG_LAUNCH_CHECK();
        const long inner = (long)F * std::max(0, g.lw[l] - 2 * g.edge) * std::max(0, g.lh[l] - 2 * g.edge);
        if (inner > 0) {
            hipLaunchKernelGGL(k_orb_nms, dim3(blocks(inner)), dim3(256), 0, s, g, l, score, cand, ccount, hist);
            MLG_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(k_orb_blur, dim3(blocks(px)), dim3(256), 0, s, g, l, pyr, blur);
        MLG_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_orb_select, dim3(F * NL), dim3(256), 0, s, g, pyr, cand, ccount, hist, sel, scount);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_orb_gather, dim3(blocks(F)), dim3(256), 0, s, g, scount, kstart, counts);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_orb_describe, dim3(blocks((long)F * max_kp)), dim3(256), 0, s, g, pyr, blur, sel, scount,
                       kstart, counts, pattern, keypoints, responses, angles, levels, descriptors);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

size_t mlg_orb_match_workspace_bytes(int P, int max_kp) {
    if (P <= 0 || max_kp <= 0) return 0;
    return (size_t)a256((long)4 * P * max_kp * 4);
}

int mlg_orb_match(const uint8_t* descriptors, const int32_t* counts, int max_kp, const int32_t* pair_a,
                  const int32_t* pair_b, int P, void* ws, size_t ws_bytes, int32_t* query_idx, int32_t* train_idx,
                  int32_t* distance, int32_t* nmatch, void* stream) {
    if (P <= 0) return MLG_OK;
    if (max_kp <= 0 || !descriptors || !counts || !pair_a || !pair_b || P > 65535) return MLG_EINVAL;
    if (!ws || ws_bytes < mlg_orb_match_workspace_bytes(P, max_kp)) return MLG_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    int* best = (int*)ws;
    int* bdist = best + (long)2 * P * max_kp;
    const dim3 grid((unsigned)((max_kp + 255) / 256), (unsigned)P);
    for (int dir = 0; dir < 2; ++dir) {
        hipLaunchKernelGGL(k_orb_nn, grid, dim3(256), 0, s, descriptors, counts, max_kp, pair_a, pair_b, dir, best,
                           bdist);
        MLG_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_orb_cross, dim3((unsigned)P), dim3(256), 0, s, counts, max_kp, pair_a, P, best, bdist,
                       query_idx, train_idx, distance, nmatch);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

}  // extern "C"
