/*
 * CPU oracle for the ORB + BFMatcher fallback matcher (TEST INFRASTRUCTURE ONLY -- see
 * oracle/__init__.py).
 *
 * Reference: LightGlue._load_fallback / _detect_and_match_fallback,
 * scripts/semantic_gating/geometric_verification.py:244-248 and 314-350:
 *   cv2.cvtColor(BGR2GRAY); cv2.ORB_create(nfeatures=max_keypoints).detectAndCompute;
 *   cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match; sorted by distance;
 *   confidence = 1 - distance / max distance.
 * OpenCV is not installed here, so this is a restatement of OpenCV 4.x's published ORB
 * (orb.cpp: scale pyramid by resize(..., INTER_LINEAR_EXACT), FAST-9 with 3x3
 * non-maximum suppression, edge-threshold border filter, retainBest by FAST score (2n,
 * ties kept), Harris response (block 7, k 0.04), retainBest by Harris (n, ties kept),
 * intensity-centroid angle with the umax circle and fastAtan2, GaussianBlur(7x7,
 * sigma 2, BORDER_REFLECT_101) of each level, rBRIEF over 256 rotated point pairs) and
 * BFMatcher's cross-checked Hamming match.
 *   - INTER_LINEAR_EXACT on 8U (resize.cpp resize_bitExact / interpolationLinear): per
 *     output coordinate f = (1 / (dst / src)) * (d + 0.5) - 0.5 in binary64, i = floor f,
 *     weight of i + 1 = cvRound((f - i) * 256) (8 fractional bits, ufixedpoint16), of i
 *     = 256 minus that; coordinates left of the image take pixel 0, right of it the last
 *     pixel; horizontal sums c0 a + c1 b (16 bit), vertical (h0 c0 + h1 c1 + 2^15) >> 16.
 *   - GaussianBlur: ORB blurs a submatrix of its bordered pyramid image without
 *     BORDER_ISOLATED, which routes 8U through sepFilter2D with the float kernel (the
 *     bit-exact fixed-point path requires an isolated source); kernel =
 *     getGaussianKernel(7, 2, CV_32F) = getGaussianKernelBitExact rounded to float; row
 *     pass s = k0 x0 + k1 x1 + ... + k6 x6 (float, left to right), column pass (symmetric
 *     filter) s = k3 c + k4 (u1 + d1) + k5 (u2 + d2) + k6 (u3 + d3), cvRound (half to
 *     even), saturated to 8 bits; the level's border is REFLECT_101 (its copyMakeBorder).
 * PARITY UNPINNED against OpenCV itself; the remaining deviations (the point pattern
 * of makeRandomPattern rather than the bit_pattern_31_ table, which is not available
 * here -- loadable through MLGATE_ORB_PATTERN --; ties in retainBest ordered by
 * (response desc, y, x) where OpenCV leaves nth_element order; OpenCV's SIMD builds may
 * fuse the blur's multiply-adds, which moves a sum by <= 1 ulp before the rounding) are
 * shared with the HIP path (csrc/orb.hip), which this file pins bit for bit.
 *
 * The per-frame geometry (level sizes and scales, features per level, pattern, umax,
 * Gaussian coefficients) is computed once by the caller (mlgate/orb.py) and passed in.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CV_PI 3.1415926535897932384626433832795

/* INTER_LINEAR_EXACT weights along one axis: source index of the left tap and the
   8-bit weight of the right tap (0 where the coordinate is clamped). */
static void exact_axis(int dsize, int ssize, int *ofs, int *c1) {
    const double inv = (double)dsize / (double)ssize, scale = 1.0 / inv;
    for (int d = 0; d < dsize; ++d) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int i = (int)floor(f);
        if (i < 0 || ssize <= 1) {
            ofs[d] = 0;
            c1[d] = 0;
        } else if (i >= ssize - 1) {
            ofs[d] = ssize - 1;
            c1[d] = 0;
        } else {
            ofs[d] = i;
            c1[d] = (int)nearbyint((f - (double)i) * 256.0);
        }
    }
}

/* cv::resize(src, dst, Size(DW, DH), 0, 0, INTER_LINEAR_EXACT), one 8-bit channel. */
void orc_resize_exact_u8(const uint8_t *src, int H, int W, uint8_t *dst, int DH, int DW) {
    int *xo = (int *)malloc(sizeof(int) * DW), *xc = (int *)malloc(sizeof(int) * DW);
    int *yo = (int *)malloc(sizeof(int) * DH), *yc = (int *)malloc(sizeof(int) * DH);
    exact_axis(DW, W, xo, xc);
    exact_axis(DH, H, yo, yc);
    for (int y = 0; y < DH; ++y) {
        const int y0 = yo[y], y1 = y0 + 1 < H ? y0 + 1 : y0;
        const uint32_t cy1 = (uint32_t)yc[y], cy0 = 256u - cy1;
        for (int x = 0; x < DW; ++x) {
            const int x0 = xo[x], x1 = x0 + 1 < W ? x0 + 1 : x0;
            const uint32_t cx1 = (uint32_t)xc[x], cx0 = 256u - cx1;
            const uint32_t h0 = cx0 * src[(size_t)y0 * W + x0] + cx1 * src[(size_t)y0 * W + x1];
            const uint32_t h1 = cx0 * src[(size_t)y1 * W + x0] + cx1 * src[(size_t)y1 * W + x1];
            dst[(size_t)y * DW + x] = (uint8_t)((h0 * cy0 + h1 * cy1 + 32768u) >> 16);
        }
    }
    free(xo);
    free(xc);
    free(yo);
    free(yc);
}

typedef struct {
    int x, y, level;
    float resp;
} Cand;

static const int CIRCLE[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                  {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

/* FAST-9 score (0 = not a corner): the largest threshold t' for which 9 contiguous
   circle pixels are all > v + t' or all < v - t' (OpenCV cornerScore<16>), given that
   the pixel passes at threshold t. */
static int fast_score(const uint8_t *img, int W, int x, int y, int t) {
    const int v = img[y * W + x];
    int d[16];
    for (int k = 0; k < 16; ++k) d[k] = img[(y + CIRCLE[k][1]) * W + x + CIRCLE[k][0]] - v;
    int best_b = -1, best_d = -1; /* max over arcs of min(p - v) / min(v - p) */
    for (int k = 0; k < 16; ++k) {
        int mb = 1 << 20, md = 1 << 20;
        for (int j = 0; j < 9; ++j) {
            const int e = d[(k + j) & 15];
            if (e < mb) mb = e;
            if (-e < md) md = -e;
        }
        if (mb > best_b) best_b = mb;
        if (md > best_d) best_d = md;
    }
    const int m = best_b > best_d ? best_b : best_d;
    return m > t ? m - 1 : 0;
}

static int cmp_cand(const void *pa, const void *pb) {
    const Cand *a = (const Cand *)pa, *b = (const Cand *)pb;
    if (a->resp != b->resp) return a->resp > b->resp ? -1 : 1;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    return a->x < b->x ? -1 : (a->x > b->x);
}

static float harris(const uint8_t *img, int W, int x, int y) {
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j) {
            const uint8_t *p = img + (y - 3 + i) * W + (x - 3 + j);
            const int ix = (p[1] - p[-1]) * 2 + (p[-W + 1] - p[-W - 1]) + (p[W + 1] - p[W - 1]);
            const int iy = (p[W] - p[-W]) * 2 + (p[W - 1] - p[-W - 1]) + (p[W + 1] - p[-W + 1]);
            a += ix * ix;
            b += iy * iy;
            c += ix * iy;
        }
    const float scale = 1.f / ((1 << 2) * 7 * 255.f);
    const float s4 = scale * scale * scale * scale;
    const float A = (float)a, B = (float)b, C = (float)c;
    return ((A * B - C * C) - (0.04f * (A + B)) * (A + B)) * s4;
}

/* OpenCV fastAtan2 (degrees, [0, 360)). */
static float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / CV_PI), p3 = -0.3258083974640975f * (float)(180 / CV_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / CV_PI), p7 = -0.04432655554792128f * (float)(180 / CV_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

static float ic_angle(const uint8_t *img, int W, int x, int y, const int *umax) {
    const uint8_t *center = img + y * W + x;
    int m01 = 0, m10 = 0;
    for (int u = -15; u <= 15; ++u) m10 += u * center[u];
    for (int v = 1; v <= 15; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = center[u + v * W], vm = center[u - v * W];
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

static int refl(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

void orc_gauss7(const uint8_t *src, int H, int W, const float *k, uint8_t *dst) {
    float *h = (float *)malloc(sizeof(float) * H * W);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float s = k[0] * (float)src[y * W + refl(x - 3, W)];
            for (int t = 1; t < 7; ++t) s = s + k[t] * (float)src[y * W + refl(x + t - 3, W)];
            h[y * W + x] = s;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float s = k[3] * h[y * W + x];
            for (int t = 1; t <= 3; ++t) s = s + k[3 + t] * (h[refl(y + t, H) * W + x] + h[refl(y - t, H) * W + x]);
            const int v = (int)nearbyintf(s);
            dst[y * W + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    free(h);
}

/* One grayscale frame -> keypoints (level-0 coordinates), levels, responses, angles,
   32-byte descriptors; returns the count (<= max_out) or -1. */
int orc_orb_detect(const uint8_t *gray, int H, int W, int nlev, const int *lw, const int *lh, const float *lscale,
                   const int *nfeat, const int *pattern, const int *umax, const float *gk, int fast_t, int edge,
                   float *kx, float *ky, int *klev, float *kresp, float *kang, uint8_t *kdesc, int max_out) {
    uint8_t **lv = (uint8_t **)calloc(nlev, sizeof(uint8_t *));
    lv[0] = (uint8_t *)malloc((size_t)H * W);
    memcpy(lv[0], gray, (size_t)H * W);
    if (lw[0] != W || lh[0] != H) return -1;
    for (int l = 1; l < nlev; ++l) {
        lv[l] = (uint8_t *)malloc((size_t)lw[l] * lh[l]);
        orc_resize_exact_u8(lv[l - 1], lh[l - 1], lw[l - 1], lv[l], lh[l], lw[l]);
    }
    int out = 0;
    for (int l = 0; l < nlev; ++l) {
        const int w = lw[l], h = lh[l];
        const uint8_t *img = lv[l];
        uint8_t *sc = (uint8_t *)calloc((size_t)w * h, 1);
        for (int y = 3; y < h - 3; ++y)
            for (int x = 3; x < w - 3; ++x) sc[y * w + x] = (uint8_t)fast_score(img, w, x, y, fast_t);
        int cap = 1024, n = 0;
        Cand *cs = (Cand *)malloc(sizeof(Cand) * cap);
        for (int y = edge; y < h - edge; ++y)
            for (int x = edge; x < w - edge; ++x) {
                const int s = sc[y * w + x];
                if (!s) continue;
                int keep = 1;
                for (int dy = -1; dy <= 1 && keep; ++dy)
                    for (int dx = -1; dx <= 1; ++dx)
                        if ((dx || dy) && sc[(y + dy) * w + x + dx] >= s) { keep = 0; break; }
                if (!keep) continue;
                if (n == cap) cs = (Cand *)realloc(cs, sizeof(Cand) * (cap *= 2));
                cs[n++] = (Cand){x, y, l, (float)s};
            }
        free(sc);
        /* retainBest(2 n_l) by FAST score, ties at the threshold kept */
        qsort(cs, n, sizeof(Cand), cmp_cand);
        int keep = n;
        if (n > 2 * nfeat[l]) {
            const float thr = cs[2 * nfeat[l] - 1].resp;
            keep = 2 * nfeat[l];
            while (keep < n && cs[keep].resp >= thr) ++keep;
        }
        for (int i = 0; i < keep; ++i) cs[i].resp = harris(img, w, cs[i].x, cs[i].y);
        qsort(cs, keep, sizeof(Cand), cmp_cand);
        int fin = keep;
        if (keep > nfeat[l]) {
            if (nfeat[l] <= 0) {
                fin = 0;
            } else {
                const float thr = cs[nfeat[l] - 1].resp;
                fin = nfeat[l];
                while (fin < keep && cs[fin].resp >= thr) ++fin;
            }
        }
        uint8_t *bl = (uint8_t *)malloc((size_t)w * h);
        orc_gauss7(img, h, w, gk, bl);
        for (int i = 0; i < fin && out < max_out; ++i, ++out) {
            const int x = cs[i].x, y = cs[i].y;
            const float ang = ic_angle(img, w, x, y, umax);
            kx[out] = (float)x * lscale[l];
            ky[out] = (float)y * lscale[l];
            klev[out] = l;
            kresp[out] = cs[i].resp;
            kang[out] = ang;
            const float rad = ang * (float)(CV_PI / 180.f);
            const float a = (float)cos((double)rad), b = (float)sin((double)rad);
            uint8_t *dd = kdesc + (size_t)out * 32;
            for (int byte = 0; byte < 32; ++byte) {
                int val = 0;
                for (int bit = 0; bit < 8; ++bit) {
                    const int *p0 = pattern + 4 * (byte * 8 + bit), *p1 = p0 + 2;
                    const int r0 = (int)lrintf((float)p0[0] * b + (float)p0[1] * a);
                    const int c0 = (int)lrintf((float)p0[0] * a - (float)p0[1] * b);
                    const int r1 = (int)lrintf((float)p1[0] * b + (float)p1[1] * a);
                    const int c1 = (int)lrintf((float)p1[0] * a - (float)p1[1] * b);
                    val |= (bl[(y + r0) * w + x + c0] < bl[(y + r1) * w + x + c1]) << bit;
                }
                dd[byte] = (uint8_t)val;
            }
        }
        free(bl);
        free(cs);
    }
    for (int l = 0; l < nlev; ++l) free(lv[l]);
    free(lv);
    return out;
}

static int hamming(const uint8_t *a, const uint8_t *b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

/* BFMatcher(NORM_HAMMING, crossCheck=True).match(d1, d2), then a stable sort by
   distance: (query, train, distance) triples; returns the count. */
int orc_bf_match(const uint8_t *d1, int n1, const uint8_t *d2, int n2, int *qi, int *ti, int *dist) {
    int *best12 = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1)), *bd12 = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1));
    int *best21 = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
    for (int i = 0; i < n1; ++i) {
        int bj = -1, bd = 1 << 30;
        for (int j = 0; j < n2; ++j) {
            const int d = hamming(d1 + 32 * i, d2 + 32 * j);
            if (d < bd) { bd = d; bj = j; }
        }
        best12[i] = bj;
        bd12[i] = bd;
    }
    for (int j = 0; j < n2; ++j) {
        int bi = -1, bd = 1 << 30;
        for (int i = 0; i < n1; ++i) {
            const int d = hamming(d2 + 32 * j, d1 + 32 * i);
            if (d < bd) { bd = d; bi = i; }
        }
        best21[j] = bi;
    }
    int n = 0;
    for (int d = 0; d <= 256; ++d)
        for (int i = 0; i < n1; ++i)
            if (best12[i] >= 0 && best21[best12[i]] == i && bd12[i] == d) {
                qi[n] = i;
                ti[n] = best12[i];
                dist[n] = d;
                ++n;
            }
    free(best12);
    free(bd12);
    free(best21);
    return n;
}
