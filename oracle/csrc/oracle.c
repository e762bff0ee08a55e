/*
 * CPU oracle kernels (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).
 *
 * Plain-C restatements of the integer/byte and order-sensitive float work on the
 * hot path, written so that the HIP product path can be checked bit-for-bit:
 *
 *   orc_resize_linear_u8  cv2.resize(img, (W', H')) with INTER_LINEAR on uint8, as
 *                         called at place_recognition.py:787 (CricaVPR._preprocess).
 *                         Restated from OpenCV's published fixed-point generic path
 *                         (11-bit coefficients, 128-bit universal-intrinsic vertical
 *                         pass + scalar tail).  cv2 is not installed here: PARITY
 *                         UNPINNED against OpenCV itself.
 *   orc_row_norms_f32     np.linalg.norm(X, axis=1) on float32 as used by
 *                         place_recognition.py:186 -- elementwise square, numpy's
 *                         pairwise summation (8-way unrolled leaves of <=128),
 *                         float32 sqrt.  Pinned bit-exact against numpy in tests.
 *   orc_knn_rows          the per-row mask / top-k / threshold / floor loop of
 *                         SemanticPlaceRecognition.find_loop_closures
 *                         (place_recognition.py:873-909) given a similarity matrix.
 *                         Tie rule: descending similarity, equal similarities by
 *                         descending index (a stable ascending argsort reversed).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- resize --- */

static int round_half_even_f(float v) { return (int)lrintf(v); } /* default FE_TONEAREST */

static int16_t sat_s16(int v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

/* Vertical-pass formula of the 128-bit SIMD loop: v_rshr_pack_u<2>(mulhi(S0>>4,b0)+mulhi(S1>>4,b1)). */
static uint8_t vres_vec(int s0, int s1, int16_t b0, int16_t b1) {
    int a0 = sat_s16(s0 >> 4), a1 = sat_s16(s1 >> 4);
    int h0 = (a0 * (int)b0) >> 16, h1 = (a1 * (int)b1) >> 16;
    int v = (int16_t)(h0 + h1); /* 16-bit lane add (wraps; cannot overflow in range) */
    v = (v + 2) >> 2;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

/* Scalar tail: FixedPtCast<int,uchar,22>. */
static uint8_t vres_scalar(int s0, int s1, int16_t b0, int16_t b1) {
    int v = (s0 * (int)b0 + s1 * (int)b1 + (1 << 21)) >> 22;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

/* First byte index of the row handled by the scalar tail of the vertical pass. */
int orc_resize_vec_end(int width_bytes) {
    int x = 0;
    for (; x <= width_bytes - 16; x += 16) {}
    for (; x < width_bytes - 8; x += 8) {}
    return x;
}

/* Per-axis source index and 11-bit weights (identical rule for x and y). */
static void axis_tab(int ssize, int dsize, int *ofs, int16_t *w0, int16_t *w1) {
    double inv_scale = (double)dsize / ssize;
    double scale = 1.0 / inv_scale;
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)floorf(f);
        f -= (float)s;
        if (s < 0) { f = 0.f; s = 0; }
        if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
        ofs[d] = s;
        w0[d] = sat_s16(round_half_even_f((1.f - f) * 2048.f));
        w1[d] = sat_s16(round_half_even_f(f * 2048.f));
    }
}

/* src: H x W x C uint8 (row-major, C in {1,3,4}); dst: DH x DW x C uint8. */
int orc_resize_linear_u8(const uint8_t *src, int H, int W, int C, uint8_t *dst, int DH, int DW) {
    if (H < 1 || W < 1 || DH < 1 || DW < 1 || C < 1) return -1;
    int *xofs = (int *)malloc(sizeof(int) * DW), *yofs = (int *)malloc(sizeof(int) * DH);
    int16_t *ax0 = (int16_t *)malloc(2 * DW), *ax1 = (int16_t *)malloc(2 * DW);
    int16_t *by0 = (int16_t *)malloc(2 * DH), *by1 = (int16_t *)malloc(2 * DH);
    int *row0 = (int *)malloc(sizeof(int) * DW * C), *row1 = (int *)malloc(sizeof(int) * DW * C);
    axis_tab(W, DW, xofs, ax0, ax1);
    axis_tab(H, DH, yofs, by0, by1);
    /* The y table's clamp never changes a weight in the generic path: source rows
       are clipped instead.  Recompute y weights without the clamp to match that. */
    {
        double scale = 1.0 / ((double)DH / H);
        for (int d = 0; d < DH; ++d) {
            float f = (float)((d + 0.5) * scale - 0.5);
            int s = (int)floorf(f);
            f -= (float)s;
            yofs[d] = s;
            by0[d] = sat_s16(round_half_even_f((1.f - f) * 2048.f));
            by1[d] = sat_s16(round_half_even_f(f * 2048.f));
        }
    }
    const int wb = DW * C, vend = orc_resize_vec_end(wb);
    for (int dy = 0; dy < DH; ++dy) {
        int sy0 = yofs[dy], sy1 = yofs[dy] + 1;
        sy0 = sy0 < 0 ? 0 : (sy0 > H - 1 ? H - 1 : sy0);
        sy1 = sy1 < 0 ? 0 : (sy1 > H - 1 ? H - 1 : sy1);
        const uint8_t *S0 = src + (size_t)sy0 * W * C, *S1 = src + (size_t)sy1 * W * C;
        for (int dx = 0; dx < DW; ++dx) {
            int sx = xofs[dx];
            int sx1 = sx + 1 < W ? sx + 1 : sx; /* weight is 0 there anyway */
            for (int c = 0; c < C; ++c) {
                row0[dx * C + c] = S0[sx * C + c] * ax0[dx] + S0[sx1 * C + c] * ax1[dx];
                row1[dx * C + c] = S1[sx * C + c] * ax0[dx] + S1[sx1 * C + c] * ax1[dx];
            }
        }
        uint8_t *D = dst + (size_t)dy * wb;
        for (int x = 0; x < wb; ++x)
            D[x] = x < vend ? vres_vec(row0[x], row1[x], by0[dy], by1[dy])
                            : vres_scalar(row0[x], row1[x], by0[dy], by1[dy]);
    }
    free(xofs); free(yofs); free(ax0); free(ax1); free(by0); free(by1); free(row0); free(row1);
    return 0;
}

/* ------------------------------------------------------- numpy row norms --- */

/* numpy's pairwise_sum for float32 (umath loops_utils pairwise sum, PW_BLOCKSIZE 128). */
static float pairwise_sum_f32(const float *a, long n) {
    if (n < 8) {
        float res = -0.0f; /* numpy starts its short-loop reduction from -0.0 */
        for (long i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum_f32(a, n2) + pairwise_sum_f32(a + n2, n - n2);
    }
}

int orc_row_norms_f32(const float *X, long N, long D, float *norms) {
    float *sq = (float *)malloc(sizeof(float) * (D > 0 ? D : 1));
    for (long i = 0; i < N; ++i) {
        const float *x = X + i * D;
        for (long j = 0; j < D; ++j) {
            volatile float p = x[j] * x[j]; /* no contraction: numpy squares first */
            sq[j] = p;
        }
        /* numpy's reduction iterator hands the inner loop at most 8192 elements
           (default ufunc buffer size); chunk results accumulate sequentially. */
        float acc = 0.0f;
        for (long c0 = 0; c0 < D; c0 += 8192) {
            long n = D - c0 < 8192 ? D - c0 : 8192;
            acc = c0 == 0 ? pairwise_sum_f32(sq, n) : acc + pairwise_sum_f32(sq + c0, n);
        }
        norms[i] = sqrtf(acc);
    }
    free(sq);
    return 0;
}

/* ------------------------------------------------------------- kNN rows --- */

/* Order used for top-k: larger similarity first; ties broken by larger index. */
static int before(float va, int ia, float vb, int ib) { return va > vb || (va == vb && ia > ib); }

/*
 * S: [Q, N] similarities of query rows q0..q0+Q-1 against all N descriptors.
 * Emits, per row, up to k matches with sim >= thr (masked entries never emitted).
 * idx/sim/valid: [Q, k]; count: [Q].
 */
int orc_knn_rows(const float *S, int Q, int N, int q0, const double *t, const int64_t *floor,
                 const uint8_t *has_floor, double min_gap, float thr, int k, int gating,
                 int32_t *idx, float *sim, uint8_t *valid, int32_t *count) {
    int *best = (int *)malloc(sizeof(int) * (k > 0 ? k : 1));
    for (int r = 0; r < Q; ++r) {
        const int i = q0 + r;
        const float *row = S + (size_t)r * N;
        int nb = 0;
        for (int j = 0; j < N; ++j) {
            if (fabs(t[j] - t[i]) < min_gap) continue;
            float v = row[j];
            if (nb < k) {
                int p = nb++;
                while (p > 0 && before(v, j, row[best[p - 1]], best[p - 1])) { best[p] = best[p - 1]; --p; }
                best[p] = j;
            } else if (k > 0 && before(v, j, row[best[k - 1]], best[k - 1])) {
                int p = k - 1;
                while (p > 0 && before(v, j, row[best[p - 1]], best[p - 1])) { best[p] = best[p - 1]; --p; }
                best[p] = j;
            }
        }
        int c = 0;
        for (int p = 0; p < nb; ++p) {
            int j = best[p];
            float v = row[j];
            if (v < thr) continue;
            idx[(size_t)r * k + c] = j;
            sim[(size_t)r * k + c] = v;
            uint8_t ok = 1;
            if (gating && has_floor[i] && has_floor[j]) ok = floor[i] == floor[j];
            valid[(size_t)r * k + c] = ok;
            ++c;
        }
        count[r] = c;
    }
    free(best);
    return 0;
}
