/* OpenCV's findEssentialMat(RANSAC) restated in C -- test infrastructure only.
 *
 * A compiled twin of oracle/geometry.py cv_ransac (K given) and five_point, for checks
 * that need the OpenCV-sequenced RANSAC on tens of thousands of pairs (a whole bench
 * step's verified pairs; the numpy restatement takes seconds per pair).  Same algorithm,
 * same sample stream, same acceptance rule:
 *   * points normalised by K, threshold thr / ((fx + fy) / 2), float32 Sampson error
 *     against float32(t^2) (EMEstimatorCallback::computeError);
 *   * cv::RNG((uint64)-1) multiply-with-carry, getSubset's duplicate redraw;
 *   * a model replaces the best iff its inlier count exceeds max(best, 4), and every
 *     replacement shrinks the budget by RANSACUpdateNumIters (cvRound = rint);
 *   * 5-point solver as geometry.py states it (Li & Hartley hidden-variable resultant):
 *     4-dim null space of the 5x9 epipolar design matrix, the 10 cubic constraints
 *     det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0, det C(z) sampled at the 11th roots of
 *     unity and inverse-DFT'd to its degree-10 coefficients, real roots, (x, y) from the
 *     null vector of C(z), E normalised to unit Frobenius norm.
 * Linear algebra differs from numpy / LAPACK in rounding only (Householder null space
 * instead of an SVD basis, Aberth roots instead of companion eigenvalues, one-sided
 * Jacobi null vectors); tests/test_oracle_geometry.py pins this file against the numpy
 * restatement (identical inlier counts on seeded geometry and on real match sets).
 * Reference call site: scripts/semantic_gating/geometric_verification.py:128-146. */
#define _GNU_SOURCE
#include <complex.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef double poly3[4][4][4]; /* coefficient of x^a y^b z^c, a + b + c <= 3 */

static void pmul(poly3 out, poly3 a, poly3 b) {
    memset(out, 0, sizeof(poly3));
    for (int a0 = 0; a0 < 4; a0++)
        for (int a1 = 0; a0 + a1 < 4; a1++)
            for (int a2 = 0; a0 + a1 + a2 < 4; a2++) {
                double ca = a[a0][a1][a2];
                if (ca == 0.0) continue;
                for (int b0 = 0; a0 + b0 < 4; b0++)
                    for (int b1 = 0; a0 + a1 + b0 + b1 < 4; b1++)
                        for (int b2 = 0; a0 + a1 + a2 + b0 + b1 + b2 < 4; b2++)
                            out[a0 + b0][a1 + b1][a2 + b2] += ca * b[b0][b1][b2];
            }
}

static void padd(poly3 out, poly3 a, double s) { /* out += s * a */
    for (int i = 0; i < 64; i++) (&out[0][0][0])[i] += s * (&a[0][0][0])[i];
}

/* null space of the 5x9 design matrix: Householder QR of A^T (9x5), Q's last 4 columns */
static void null4(const double A[5][9], double N[4][9]) {
    double M[9][5], Q[9][9];
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 5; j++) M[i][j] = A[j][i];
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) Q[i][j] = (i == j);
    for (int j = 0; j < 5; j++) {
        double nrm = 0.0;
        for (int i = j; i < 9; i++) nrm += M[i][j] * M[i][j];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        double v[9] = {0};
        double alpha = M[j][j] > 0 ? -nrm : nrm;
        for (int i = j; i < 9; i++) v[i] = M[i][j];
        v[j] -= alpha;
        double vv = 0.0;
        for (int i = j; i < 9; i++) vv += v[i] * v[i];
        if (vv == 0.0) continue;
        for (int c = j; c < 5; c++) { /* M = H M */
            double d = 0.0;
            for (int i = j; i < 9; i++) d += v[i] * M[i][c];
            d = 2.0 * d / vv;
            for (int i = j; i < 9; i++) M[i][c] -= d * v[i];
        }
        for (int r = 0; r < 9; r++) { /* Q = Q H */
            double d = 0.0;
            for (int i = j; i < 9; i++) d += Q[r][i] * v[i];
            d = 2.0 * d / vv;
            for (int i = j; i < 9; i++) Q[r][i] -= d * v[i];
        }
    }
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 9; i++) N[k][i] = Q[i][5 + k];
}

static double complex cdet10(double complex A[10][10]) {
    double complex det = 1.0;
    for (int c = 0; c < 10; c++) {
        int p = c;
        for (int r = c + 1; r < 10; r++)
            if (fabs(creal(A[r][c])) + fabs(cimag(A[r][c])) > fabs(creal(A[p][c])) + fabs(cimag(A[p][c]))) p = r;
        if (A[p][c] == 0.0) return 0.0;
        if (p != c) {
            for (int j = 0; j < 10; j++) {
                double complex t = A[c][j];
                A[c][j] = A[p][j];
                A[p][j] = t;
            }
            det = -det;
        }
        det *= A[c][c];
        for (int r = c + 1; r < 10; r++) {
            double complex f = A[r][c] / A[c][c];
            for (int j = c; j < 10; j++) A[r][j] -= f * A[c][j];
        }
    }
    return det;
}

/* roots of c[0] + c[1] z + ... + c[deg] z^deg (np.roots: leading / trailing exact zeros
 * stripped, trailing ones give roots at 0); Aberth-Ehrlich iteration + Newton polish */
static int poly_roots(const double *c_in, int deg, double complex *roots) {
    double c[16];
    memcpy(c, c_in, sizeof(double) * (deg + 1));
    while (deg > 0 && c[deg] == 0.0) deg--;
    int nz = 0, nr = 0;
    while (nz < deg && c[nz] == 0.0) nz++;
    for (int i = 0; i < nz; i++) roots[nr++] = 0.0;
    const double *p = c + nz;
    int n = deg - nz;
    if (n <= 0) return nr;
    /* initial points: a circle of the geometric-mean radius, off the real axis */
    double rad = pow(fabs(p[0] / p[n]), 1.0 / n);
    if (!(rad > 0.0) || !isfinite(rad)) rad = 1.0;
    double complex z[16];
    for (int i = 0; i < n; i++) z[i] = rad * cexp(I * (2.0 * M_PI * i / n + 0.4));
    int done[16] = {0}, left = n;
    for (int it = 0; it < 200 && left > 0; it++) {
        for (int i = 0; i < n; i++) {
            if (done[i]) continue;
            double complex f = p[n], d = 0.0;
            for (int k = n - 1; k >= 0; k--) {
                d = d * z[i] + f;
                f = f * z[i] + p[k];
            }
            if (f == 0.0) {
                done[i] = 1;
                left--;
                continue;
            }
            double complex ratio = f / d, s = 0.0;
            for (int j = 0; j < n; j++)
                if (j != i) s += 1.0 / (z[i] - z[j]);
            double complex w = ratio / (1.0 - ratio * s);
            z[i] -= w;
            if (cabs(w) <= 1e-14 * fmax(1e-300, cabs(z[i]))) {
                done[i] = 1;
                left--;
            }
        }
    }
    for (int i = 0; i < n; i++) { /* Newton polish */
        for (int it = 0; it < 3; it++) {
            double complex f = p[n], d = 0.0;
            for (int k = n - 1; k >= 0; k--) {
                d = d * z[i] + f;
                f = f * z[i] + p[k];
            }
            if (d == 0.0 || f == 0.0) break;
            z[i] -= f / d;
        }
        roots[nr++] = z[i];
    }
    return nr;
}

/* null vector of a real 10x10 of rank 9: Householder QR with column pivoting of A^T
 * (the rows of A, largest remaining norm first); the last column of Q is orthogonal to
 * the 9 pivot rows, i.e. spans the null space (geometry.py takes the SVD's last right
 * singular vector: the same direction up to sign and rounding) */
static void null_vec10(double A[10][10], double out[10]) {
    double M[10][10], Q[10][10];
    for (int i = 0; i < 10; i++)
        for (int j = 0; j < 10; j++) {
            M[i][j] = A[j][i]; /* column j of M = row j of A */
            Q[i][j] = (i == j);
        }
    for (int j = 0; j < 9; j++) {
        int piv = j;
        double best = -1.0;
        for (int c = j; c < 10; c++) {
            double nn = 0.0;
            for (int i = j; i < 10; i++) nn += M[i][c] * M[i][c];
            if (nn > best) {
                best = nn;
                piv = c;
            }
        }
        if (piv != j)
            for (int i = 0; i < 10; i++) {
                double t = M[i][j];
                M[i][j] = M[i][piv];
                M[i][piv] = t;
            }
        double nrm = sqrt(best);
        if (nrm == 0.0) continue;
        double v[10] = {0};
        double alpha = M[j][j] > 0 ? -nrm : nrm;
        for (int i = j; i < 10; i++) v[i] = M[i][j];
        v[j] -= alpha;
        double vv = 0.0;
        for (int i = j; i < 10; i++) vv += v[i] * v[i];
        if (vv == 0.0) continue;
        for (int c = j; c < 10; c++) {
            double d = 0.0;
            for (int i = j; i < 10; i++) d += v[i] * M[i][c];
            d = 2.0 * d / vv;
            for (int i = j; i < 10; i++) M[i][c] -= d * v[i];
        }
        for (int r = 0; r < 10; r++) {
            double d = 0.0;
            for (int i = j; i < 10; i++) d += Q[r][i] * v[i];
            d = 2.0 * d / vv;
            for (int i = j; i < 10; i++) Q[r][i] -= d * v[i];
        }
    }
    for (int i = 0; i < 10; i++) out[i] = Q[i][9];
}

static const int XY[10][2] = {{3, 0}, {2, 1}, {1, 2}, {0, 3}, {2, 0}, {1, 1}, {0, 2}, {1, 0}, {0, 1}, {0, 0}};

/* all real essential matrices through 5 normalised correspondences (row-major 3x3, unit
 * Frobenius); returns their number (<= 10).  geometry.py five_point. */
int orc_five_point(const double *q1, const double *q2, double *E_out) {
    double A[5][9], N[4][9];
    for (int i = 0; i < 5; i++) {
        double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double row[9] = {x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, 1.0};
        memcpy(A[i], row, sizeof(row));
    }
    null4(A, N);
    poly3 E[9];
    memset(E, 0, sizeof(E));
    for (int k = 0; k < 9; k++) {
        E[k][1][0][0] = N[0][k];
        E[k][0][1][0] = N[1][k];
        E[k][0][0][1] = N[2][k];
        E[k][0][0][0] = N[3][k];
    }
    poly3 eqs[10], t1, t2, t3;
    memset(eqs, 0, sizeof(eqs));
    static const int DT[3][6] = {{1, 0, 4, 8, 5, 7}, {-1, 1, 3, 8, 5, 6}, {1, 2, 3, 7, 4, 6}};
    for (int r = 0; r < 3; r++) {
        const int *d = DT[r];
        pmul(t1, E[d[2]], E[d[3]]);
        pmul(t2, E[d[4]], E[d[5]]);
        padd(t1, t2, -1.0);
        pmul(t3, E[d[1]], t1);
        padd(eqs[0], t3, (double)d[0]);
    }
    static poly3 EEt[3][3];
    memset(EEt, 0, sizeof(EEt));
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            for (int k = 0; k < 3; k++) {
                pmul(t1, E[i * 3 + k], E[j * 3 + k]);
                padd(EEt[i][j], t1, 1.0);
            }
    poly3 tr;
    memset(tr, 0, sizeof(tr));
    padd(tr, EEt[0][0], 1.0);
    padd(tr, EEt[1][1], 1.0);
    padd(tr, EEt[2][2], 1.0);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            poly3 *acc = &eqs[1 + i * 3 + j];
            for (int k = 0; k < 3; k++) {
                memcpy(t2, EEt[i][k], sizeof(poly3));
                if (i == k) padd(t2, tr, -0.5);
                pmul(t1, t2, E[k * 3 + j]);
                padd(*acc, t1, 1.0);
            }
        }
    /* det C(z) at the 11th roots of unity -> degree-10 coefficients */
    static double complex tw[11];
    static int tw_ready = 0;
    if (!tw_ready) {
        for (int s = 0; s < 11; s++) tw[s] = cexp(2.0 * M_PI * I * s / 11.0);
        tw_ready = 1;
    }
    double complex vals[11];
    for (int s = 0; s < 11; s++) {
        double complex w = tw[s], C[10][10];
        for (int r = 0; r < 10; r++)
            for (int col = 0; col < 10; col++) {
                int a = XY[col][0], b = XY[col][1];
                double complex v = 0.0, zp = 1.0;
                for (int c = 0; c < 4 - a - b; c++) {
                    v += eqs[r][a][b][c] * zp;
                    zp *= w;
                }
                C[r][col] = v;
            }
        vals[s] = cdet10(C);
    }
    double coef[11];
    for (int j = 0; j < 11; j++) {
        double complex acc = 0.0;
        for (int s = 0; s < 11; s++) acc += vals[s] * conj(tw[(j * s) % 11]);
        coef[j] = creal(acc) / 11.0;
    }
    double complex roots[16];
    int nr = poly_roots(coef, 10, roots);
    int out = 0;
    for (int ri = 0; ri < nr; ri++) {
        double complex zc = roots[ri];
        if (fabs(cimag(zc)) > 1e-8 * fmax(1.0, cabs(zc))) continue;
        double z = creal(zc), C[10][10], m[10];
        for (int r = 0; r < 10; r++)
            for (int col = 0; col < 10; col++) {
                int a = XY[col][0], b = XY[col][1];
                double v = 0.0, zp = 1.0;
                for (int c = 0; c < 4 - a - b; c++) {
                    v += eqs[r][a][b][c] * zp;
                    zp *= z;
                }
                C[r][col] = v;
            }
        null_vec10(C, m);
        if (fabs(m[9]) < 1e-300) continue;
        double x = m[7] / m[9], y = m[8] / m[9], Ev[9], nrm = 0.0;
        for (int k = 0; k < 9; k++) {
            Ev[k] = x * N[0][k] + y * N[1][k] + z * N[2][k] + N[3][k];
            nrm += Ev[k] * Ev[k];
        }
        nrm = sqrt(nrm);
        for (int k = 0; k < 9; k++) E_out[out * 9 + k] = Ev[k] / nrm;
        out++;
    }
    return out;
}

typedef struct {
    uint64_t state;
} cvrng;

static uint32_t rng_next(cvrng *r) {
    r->state = (uint64_t)(uint32_t)r->state * 4164903690ULL + (r->state >> 32);
    return (uint32_t)r->state;
}

static int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmin(fmax(p, 0.0), 1.0);
    ep = fmin(fmax(ep, 0.0), 1.0);
    double num = fmax(1.0 - p, DBL_MIN);
    double denom = 1.0 - pow(1.0 - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

static int sampson_count(const double *E, const double *p1, const double *p2, int n, float t2, uint8_t *mask) {
    int g = 0;
    for (int i = 0; i < n; i++) {
        double x1 = p1[2 * i], y1 = p1[2 * i + 1], x2 = p2[2 * i], y2 = p2[2 * i + 1];
        double a0 = E[0] * x1 + E[1] * y1 + E[2], a1 = E[3] * x1 + E[4] * y1 + E[5], a2 = E[6] * x1 + E[7] * y1 + E[8];
        double b0 = x2 * E[0] + y2 * E[3] + E[6], b1 = x2 * E[1] + y2 * E[4] + E[7];
        double r = x2 * a0 + y2 * a1 + a2;
        float err = (float)(r * r / (a0 * a0 + a1 * a1 + b0 * b0 + b1 * b1));
        int in = err <= t2;
        if (mask) mask[i] = (uint8_t)in;
        g += in;
    }
    return g;
}

/* cv2.findEssentialMat(k1, k2, K, RANSAC, prob, threshold) -> inlier count; mask [n] and
 * the best model (row-major 3x3) when non-null.  geometry.py cv_ransac (K given). */
int orc_essential_ransac(const float *k1, const float *k2, int n, const double *K, double thr, double conf,
                         int max_iters, uint8_t *mask_out, double *E_best) {
    enum { M = 5 };
    if (mask_out) memset(mask_out, 0, (size_t)n);
    if (n < M) return 0;
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double p1[2 * 2048 + 16], p2[2 * 2048 + 16];
    if (n > 2048 + 8) return -1;
    for (int i = 0; i < n; i++) {
        p1[2 * i] = ((double)k1[2 * i] - cx) / fx;
        p1[2 * i + 1] = ((double)k1[2 * i + 1] - cy) / fy;
        p2[2 * i] = ((double)k2[2 * i] - cx) / fx;
        p2[2 * i + 1] = ((double)k2[2 * i + 1] - cy) / fy;
    }
    double t = thr / ((fx + fy) / 2.0);
    float t2 = (float)(t * t);
    double Es[90], q1[10], q2[10];
    uint8_t cur[2048 + 16];
    if (n == M) {
        int ns = orc_five_point(p1, p2, Es);
        if (!ns) return 0;
        if (mask_out) memset(mask_out, 1, (size_t)n);
        if (E_best) memcpy(E_best, Es, sizeof(double) * 9);
        return n;
    }
    cvrng rng = {~0ULL};
    int niters = max_iters, max_good = 0;
    for (int it = 0; it < niters; it++) {
        int idx[M];
        for (int i = 0; i < M; i++) {
            int v, dup;
            do {
                v = (int)(rng_next(&rng) % (uint32_t)n);
                dup = 0;
                for (int j = 0; j < i; j++) dup |= idx[j] == v;
            } while (dup);
            idx[i] = v;
        }
        for (int i = 0; i < M; i++) {
            q1[2 * i] = p1[2 * idx[i]];
            q1[2 * i + 1] = p1[2 * idx[i] + 1];
            q2[2 * i] = p2[2 * idx[i]];
            q2[2 * i + 1] = p2[2 * idx[i] + 1];
        }
        int ns = orc_five_point(q1, q2, Es);
        for (int s = 0; s < ns; s++) {
            int g = sampson_count(Es + 9 * s, p1, p2, n, t2, cur);
            if (g > (max_good > M - 1 ? max_good : M - 1)) {
                max_good = g;
                if (mask_out) memcpy(mask_out, cur, (size_t)n);
                if (E_best) memcpy(E_best, Es + 9 * s, sizeof(double) * 9);
                niters = update_num_iters(conf, (double)(n - g) / n, M, niters);
            }
        }
    }
    return max_good;
}
