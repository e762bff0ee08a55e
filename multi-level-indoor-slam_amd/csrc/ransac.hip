// Batched epipolar RANSAC + relative pose for geometric verification.
//
// Replaces, for a batch of candidate pairs at once, the OpenCV calls of
// BaseFeatureMatcher.verify_geometric_consistency / estimate_relative_pose
// (geometric_verification.py:104-188):
//   K given : cv2.findEssentialMat(k1, k2, K, RANSAC, prob 0.999, threshold) -- points
//             normalised by K, threshold / ((fx + fy) / 2), 5-point minimal solver,
//             Sampson error, inlier iff (float)err <= (float)thr^2; then
//             cv2.recoverPose(E, k1[in], k2[in], K) (4-fold decomposition, cheirality
//             with depth < 50, ties in the order (R1,t), (R2,t), (R1,-t), (R2,-t)).
//   K absent: cv2.findFundamentalMat(k1, k2, FM_RANSAC, threshold, 0.999) -- 7-point
//             solver, error max(d1^2, d2^2) of the two point-to-epiline distances in
//             pixels; 7 points: the 7-point model directly; 8..14 points: LMedS (as
//             OpenCV does below 15 points); fewer than 7: no model.
// RANSAC follows OpenCV's RANSACPointSetRegistrator::run (calib3d/ptsetreg.cpp) step
// for step, restated so its sequential control flow runs in parallel:
//   * the minimal samples are OpenCV's: cv::RNG((uint64)-1) (multiply-with-carry,
//     coefficient 4164903690), getSubset's duplicate redraw and, for F, checkSubset's
//     collinearity test (haveCollinearPoints, FLT_EPSILON) -- one thread per pair
//     replays the RNG stream and writes the H = maxIters subsets;
//   * every subset is solved and scored in parallel (one thread per hypothesis);
//   * one thread per pair then scans the hypotheses in iteration order exactly as
//     the sequential loop would: a model replaces the best iff its inlier count
//     exceeds max(best, modelPoints - 1), and each replacement shrinks the iteration
//     budget by RANSACUpdateNumIters(0.999, outlier ratio, modelPoints, niters), so
//     hypotheses past the adaptive stop are ignored;
//   * no model when no count exceeded modelPoints - 1 (OpenCV's maxGoodCount == 0).
// The inlier count therefore equals OpenCV's for the same matches; only the order of
// several solutions of one sample (solver-specific) can pick a different model among
// equal counts.  LMedS (F, 8..14 matches) keeps a seeded counter-based sample stream.
//
// Pipeline (one pair = one segment of the flat match arrays):
//   k_ransac_prep    : normalised double coordinates (+ Hartley transforms for F)
//   k_ransac_subsets : one thread per pair: OpenCV's sample stream
//   k_ransac_hyp     : one thread per hypothesis: solve (<= 10 models)
//   k_ransac_score   : one thread per hypothesis: inlier count (or LMedS median) of
//                      each model over the pair's points, staged in LDS
//   (hyp / hyp5 / score run in two rounds: hypotheses [0, 256) of every pair, then
//   k_ransac_probe replays the sequential scan over them and only the pairs whose
//   adaptive stop lies beyond get hypotheses [256, H))
//   k_ransac_select  : one workgroup per pair: OpenCV's sequential best-model scan,
//                      inlier mask
//   k_recover_pose   : one workgroup per pair: E -> [R|t] by cheirality on the inliers
#include "common.h"
#include "kernels.h"

// Values that feed a branch, a root or a count come from rs_math.h, the one header the C
// twin (oracle/csrc/ransac_cv.c) includes too; this file builds with -ffp-contract=off
// (csrc/Makefile) as the twin does, so both produce the same bits (tests/test_ransac_gpu.py).
#define RS_FN __host__ __device__ static inline
#define RS_CONST static __constant__ const
#include "rs_math.h"

namespace {

#define RS_HD __host__ __device__  // solvers also build for host-side unit checks

constexpr int MAXSOL = 10;
constexpr int RS_CHUNK = 1024;  // points per LDS stage in scoring (4 doubles each = 32 KB)
constexpr int RS_ROUND1 = 256;  // hypotheses of the first round (inlier ratio >= 0.5 stops inside it)

// A hypothesis' solution count as the readers use it, clamped to [0, MAXSOL]: the solver
// kernels write every slot they own, but a slot left unwritten by a future bug (round 4:
// 5-point direct pairs) must not index past the pair's MAXSOL models and scores.
__device__ __forceinline__ int nsol_at(const int8_t* __restrict__ nsol, size_t i) {
    return min(max((int)nsol[i], 0), MAXSOL);
}

// ------------------------------------------------------------------ small linear algebra

// Null space of an m x 9 matrix (m = 5 or 7) by Gauss-Jordan elimination with partial
// pivoting; writes 9 - m basis vectors (rank-deficient samples return false).
template <int MR>
RS_HD bool null_space9(double (&A)[MR][9], double (&N)[9 - MR][9]) {
    int piv_col[MR];
    int r = 0;
    for (int c = 0; c < 9 && r < MR; ++c) {
        int best = r;
        double bv = fabs(A[r][c]);
        for (int i = r + 1; i < MR; ++i)
            if (fabs(A[i][c]) > bv) { bv = fabs(A[i][c]); best = i; }
        if (bv < 1e-12) continue;
        if (best != r)
            for (int j = 0; j < 9; ++j) { double t = A[r][j]; A[r][j] = A[best][j]; A[best][j] = t; }
        const double inv = 1.0 / A[r][c];
        for (int j = 0; j < 9; ++j) A[r][j] *= inv;
        for (int i = 0; i < MR; ++i)
            if (i != r) {
                const double f = A[i][c];
                if (f != 0.0)
                    for (int j = 0; j < 9; ++j) A[i][j] -= f * A[r][j];
            }
        piv_col[r++] = c;
    }
    if (r < MR) return false;
    bool is_piv[9] = {false, false, false, false, false, false, false, false, false};
    for (int i = 0; i < MR; ++i) is_piv[piv_col[i]] = true;
    int k = 0;
    for (int f = 0; f < 9; ++f) {
        if (is_piv[f]) continue;
        for (int j = 0; j < 9; ++j) N[k][j] = 0.0;
        N[k][f] = 1.0;
        for (int i = 0; i < MR; ++i) N[k][piv_col[i]] = -A[i][f];
        ++k;
    }
    // orthonormalise (modified Gram-Schmidt, two passes): keeps the hidden-variable
    // polynomial well conditioned (coefficients O(1), roots of moderate size)
    for (int pass = 0; pass < 2; ++pass)
        for (int a = 0; a < 9 - MR; ++a) {
            for (int q = 0; q < a; ++q) {
                double d = 0.0;
                for (int j = 0; j < 9; ++j) d += N[a][j] * N[q][j];
                for (int j = 0; j < 9; ++j) N[a][j] -= d * N[q][j];
            }
            double n2 = 0.0;
            for (int j = 0; j < 9; ++j) n2 += N[a][j] * N[a][j];
            n2 = 1.0 / sqrt(n2);
            for (int j = 0; j < 9; ++j) N[a][j] *= n2;
        }
    return true;
}

RS_HD double det3(const double* F) {
    return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) +
           F[2] * (F[3] * F[7] - F[4] * F[6]);
}

// Real roots of sum_i c[i] x^i (degree <= 10) by recursive isolation between the
// roots of the derivative, refined by safeguarded bisection / regula falsi.
RS_HD double peval(const double* c, int n, double x) {
    double v = c[n];
    for (int i = n - 1; i >= 0; --i) v = v * x + c[i];
    return v;
}

RS_HD double refine_root(const double* c, int n, double lo, double hi, double flo) {
    double fl = flo, fh = peval(c, n, hi);
    int side = 0;
    for (int it = 0; it < 100; ++it) {
        double x = (lo * fh - hi * fl) / (fh - fl);
        if (!(x > lo && x < hi)) x = 0.5 * (lo + hi);
        const double fx = peval(c, n, x);
        if (fx == 0.0) return x;
        if ((fx < 0) == (fl < 0)) {
            lo = x; fl = fx;
            if (side == -1) fh *= 0.5;
            side = -1;
        } else {
            hi = x; fh = fx;
            if (side == 1) fl *= 0.5;
            side = 1;
        }
        if (hi - lo <= 1e-14 * fmax(1.0, fabs(lo))) break;
    }
    return 0.5 * (lo + hi);
}

RS_HD int real_roots(const double* cin, int deg, double* roots) {
    double c[11];
    int n = deg;
    double mx = 0.0;
    for (int i = 0; i <= deg; ++i) { c[i] = cin[i]; mx = fmax(mx, fabs(c[i])); }
    if (mx == 0.0) return 0;
    while (n > 0 && fabs(c[n]) <= 1e-13 * mx) --n;
    if (n == 0) return 0;
    for (int i = 0; i <= n; ++i) c[i] /= c[n];
    double B = 0.0;
    for (int i = 0; i < n; ++i) B = fmax(B, fabs(c[i]));
    B += 1.0;
    // derivative chain d[k] = c^(k) / k!-scaled (monic not needed)
    double d[11][11];
    for (int i = 0; i <= n; ++i) d[0][i] = c[i];
    for (int k = 1; k < n; ++k)
        for (int i = 0; i <= n - k; ++i) d[k][i] = d[k - 1][i + 1] * (double)(i + 1);
    double crit[11];
    int ncrit = 0;
    // linear d[n-1]: root
    crit[0] = -d[n - 1][0] / d[n - 1][1];
    ncrit = 1;
    for (int k = n - 2; k >= 0; --k) {
        const int dg = n - k;
        double pts[12];
        int np = 0;
        pts[np++] = -B;
        for (int i = 0; i < ncrit; ++i)
            if (crit[i] > -B && crit[i] < B) pts[np++] = crit[i];
        pts[np++] = B;
        double nr[11];
        int nn = 0;
        double fprev = peval(d[k], dg, pts[0]);
        for (int i = 1; i < np; ++i) {
            const double f = peval(d[k], dg, pts[i]);
            if (fprev == 0.0) {
                if (nn == 0 || nr[nn - 1] != pts[i - 1]) nr[nn++] = pts[i - 1];
            } else if ((fprev < 0) != (f < 0) && f != 0.0) {
                nr[nn++] = refine_root(d[k], dg, pts[i - 1], pts[i], fprev);
            }
            fprev = f;
        }
        if (fprev == 0.0 && (nn == 0 || nr[nn - 1] != pts[np - 1])) nr[nn++] = pts[np - 1];
        ncrit = nn;
        for (int i = 0; i < nn; ++i) crit[i] = nr[i];
    }
    for (int i = 0; i < ncrit; ++i) roots[i] = crit[i];
    return ncrit;
}

// ------------------------------------------------------------------ 7-point solver
RS_HD int solve_7pt(const double (&q1)[7][2], const double (&q2)[7][2], double* Fout) {
    double A[7][9];
    for (int i = 0; i < 7; ++i) {
        const double x1 = q1[i][0], y1 = q1[i][1], x2 = q2[i][0], y2 = q2[i][1];
        A[i][0] = x2 * x1; A[i][1] = x2 * y1; A[i][2] = x2;
        A[i][3] = y2 * x1; A[i][4] = y2 * y1; A[i][5] = y2;
        A[i][6] = x1;      A[i][7] = y1;      A[i][8] = 1.0;
    }
    double Nb[2][9];
    if (!null_space9<7>(A, Nb)) return 0;
    // det(a F1 + (1 - a) F2) = cubic in a, interpolated at a = -1, 0, 1, 2
    double f[4];
    const double as[4] = {-1.0, 0.0, 1.0, 2.0};
    for (int i = 0; i < 4; ++i) {
        double F[9];
        for (int k = 0; k < 9; ++k) F[k] = as[i] * Nb[0][k] + (1.0 - as[i]) * Nb[1][k];
        f[i] = det3(F);
    }
    // Newton divided differences -> monomial coefficients
    const double d1 = f[1] - f[0], d2 = f[2] - f[1], d3 = f[3] - f[2];
    const double e1 = (d2 - d1) / 2.0, e2 = (d3 - d2) / 2.0;
    const double g = (e2 - e1) / 3.0;
    // p(a) = f0 + d1 (a+1) + e1 (a+1) a + g (a+1) a (a-1)
    double c[4];
    c[3] = g;
    c[2] = e1;
    c[1] = d1 + e1 - g;
    c[0] = f[0] + d1;
    double roots[3];
    const int nr = real_roots(c, 3, roots);
    int ns = 0;
    for (int t = 0; t < nr; ++t) {
        double* F = Fout + ns * 9;
        double nrm = 0.0;
        for (int k = 0; k < 9; ++k) {
            F[k] = roots[t] * Nb[0][k] + (1.0 - roots[t]) * Nb[1][k];
            nrm += F[k] * F[k];
        }
        if (!(nrm > 0.0)) continue;
        nrm = 1.0 / sqrt(nrm);
        for (int k = 0; k < 9; ++k) F[k] *= nrm;
        ++ns;
    }
    return ns;
}

// ------------------------------------------------------------------ errors
// Sampson error of E on normalised points (OpenCV EMEstimatorCallback::computeError).
RS_HD __forceinline__ float err_sampson(const double* E, double x1, double y1, double x2, double y2) {
    const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
    const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
    const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
    const double et0 = E[0] * x2 + E[3] * y2 + E[6];
    const double et1 = E[1] * x2 + E[4] * y2 + E[7];
    const double r = x2 * ex0 + y2 * ex1 + ex2;
    return (float)(r * r / (ex0 * ex0 + ex1 * ex1 + et0 * et0 + et1 * et1));
}

// err_sampson(E, ...) <= t2f without the division on almost every point: with
// hi = the midpoint between t2f and the next float (the largest value that still
// rounds to <= t2f, ties to even), (float)(num / den) <= t2f iff num / den < hi (or ==
// hi with an even t2f).  Points whose num clears hi * den by a relative 1e-12 are
// decided by one multiply; the rest take the exact division, so the verdict is the
// same bit for bit.
RS_HD __forceinline__ bool sampson_inlier(const double* E, double x1, double y1, double x2, double y2, float t2f,
                                          double hi) {
    const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
    const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
    const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
    const double et0 = E[0] * x2 + E[3] * y2 + E[6];
    const double et1 = E[1] * x2 + E[4] * y2 + E[7];
    const double r = x2 * ex0 + y2 * ex1 + ex2;
    const double num = r * r, den = ex0 * ex0 + ex1 * ex1 + et0 * et0 + et1 * et1;
    const double lim = hi * den;
    if (num < lim * (1.0 - 1e-12)) return true;
    if (num > lim * (1.0 + 1e-12)) return false;
    return (float)(num / den) <= t2f;
}

// max of the squared point-to-epiline distances in pixels (FMEstimatorCallback).
RS_HD __forceinline__ float err_epiline(const double* F, double x1, double y1, double x2, double y2) {
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1.0 / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1.0 / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    return (float)fmax(d1 * d1 * s1, d2 * d2 * s2);
}

RS_HD __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// cv::RNG (core/include/opencv2/core/operations.hpp): state' = (uint32)state * 4164903690
// + (state >> 32); next() = (uint32)state'; uniform(a, b) = next() % (b - a) + a.
struct CvRng {
    uint64_t state;
    RS_HD unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690ull + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    RS_HD int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a)) + a; }
};

constexpr double RANSAC_CONFIDENCE = 0.999;  // findEssentialMat / findFundamentalMat prob
constexpr int RANSAC_MAX_ATTEMPTS = 10000;   // getSubset(..., maxAttempts) in run()

// RANSACUpdateNumIters (ptsetreg.cpp), rs_math.h
RS_HD int ransac_update_iters(double p, double ep, int model_points, int max_iters) {
    return rs_update_iters(p, ep, model_points, max_iters);
}

// haveCollinearPoints (fundam.cpp) for the last of `count` selected points
RS_HD bool collinear_last(const float (*pt)[2], int count) {
    const int i = count - 1;
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)(pt[j][0] - pt[i][0]), dy1 = (double)(pt[j][1] - pt[i][1]);
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)(pt[k][0] - pt[i][0]), dy2 = (double)(pt[k][1] - pt[i][1]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= 1.1920928955078125e-07 * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

// per-pair parameters in workspace
struct PairInfo {
    int start, count, mode;  // mode: 0 none, 1 E RANSAC, 2 F RANSAC, 3 F LMedS, 4 F direct (7 pts), 5 E direct (5 pts)
    int pad;
    double thr2;          // squared threshold in the error's units
    double T1[3], T2[3];  // F: Hartley transforms (s, tx, ty): x' = s x + tx
    double Kn[4];         // E: fx, fy, cx, cy
};

// pts layout per match: [x1n, y1n, x2n, y2n] (E: K-normalised, F: Hartley-normalised);
// raw pixel copy for F scoring: [x1, y1, x2, y2]
__global__ void k_ransac_prep(const float* __restrict__ kp1, const float* __restrict__ kp2,
                              const int32_t* __restrict__ offs, const double* __restrict__ K, int k_stride, double thr,
                              PairInfo* __restrict__ info, double4* __restrict__ ptsn, double4* __restrict__ ptsr) {
    const int p = blockIdx.x;
    const int s0 = offs[p], S = offs[p + 1] - offs[p];
    __shared__ double red[4][256];
    PairInfo pi;
    pi.start = s0;
    pi.count = S;
    pi.pad = 0;
    const bool ess = K != nullptr;
    if (ess) {
        const double* Kp = K + (size_t)p * k_stride;
        const double fx = Kp[0], fy = Kp[4], cx = Kp[2], cy = Kp[5];
        pi.Kn[0] = fx; pi.Kn[1] = fy; pi.Kn[2] = cx; pi.Kn[3] = cy;
        const double t = thr / ((fx + fy) * 0.5);
        pi.thr2 = t * t;
        pi.mode = S < 5 ? 0 : (S == 5 ? 5 : 1);
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            const double x1 = kp1[2 * (s0 + i)], y1 = kp1[2 * (s0 + i) + 1];
            const double x2 = kp2[2 * (s0 + i)], y2 = kp2[2 * (s0 + i) + 1];
            ptsn[s0 + i] = make_double4((x1 - cx) / fx, (y1 - cy) / fy, (x2 - cx) / fx, (y2 - cy) / fy);
        }
        for (int j = 0; j < 3; ++j) { pi.T1[j] = 0.0; pi.T2[j] = 0.0; }
    } else {
        pi.thr2 = thr * thr;
        pi.mode = S < 7 ? 0 : (S == 7 ? 4 : (S < 15 ? 3 : 2));
        for (int j = 0; j < 4; ++j) pi.Kn[j] = 0.0;
        // Hartley normalisation: centroid + mean distance sqrt(2)
        double s[4] = {0, 0, 0, 0};
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            s[0] += kp1[2 * (s0 + i)]; s[1] += kp1[2 * (s0 + i) + 1];
            s[2] += kp2[2 * (s0 + i)]; s[3] += kp2[2 * (s0 + i) + 1];
        }
        for (int j = 0; j < 4; ++j) red[j][threadIdx.x] = s[j];
        __syncthreads();
        for (int o = blockDim.x / 2; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o)
                for (int j = 0; j < 4; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + o];
            __syncthreads();
        }
        const double inv = S > 0 ? 1.0 / S : 0.0;
        const double m1x = red[0][0] * inv, m1y = red[1][0] * inv, m2x = red[2][0] * inv, m2y = red[3][0] * inv;
        __syncthreads();
        double d[2] = {0, 0};
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            d[0] += rs_hypot(kp1[2 * (s0 + i)] - m1x, kp1[2 * (s0 + i) + 1] - m1y);
            d[1] += rs_hypot(kp2[2 * (s0 + i)] - m2x, kp2[2 * (s0 + i) + 1] - m2y);
        }
        red[0][threadIdx.x] = d[0];
        red[1][threadIdx.x] = d[1];
        __syncthreads();
        for (int o = blockDim.x / 2; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) {
                red[0][threadIdx.x] += red[0][threadIdx.x + o];
                red[1][threadIdx.x] += red[1][threadIdx.x + o];
            }
            __syncthreads();
        }
        const double md1 = red[0][0] * inv, md2 = red[1][0] * inv;
        const double sc1 = md1 > 0 ? M_SQRT2 / md1 : 1.0, sc2 = md2 > 0 ? M_SQRT2 / md2 : 1.0;
        pi.T1[0] = sc1; pi.T1[1] = -sc1 * m1x; pi.T1[2] = -sc1 * m1y;
        pi.T2[0] = sc2; pi.T2[1] = -sc2 * m2x; pi.T2[2] = -sc2 * m2y;
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            const double x1 = kp1[2 * (s0 + i)], y1 = kp1[2 * (s0 + i) + 1];
            const double x2 = kp2[2 * (s0 + i)], y2 = kp2[2 * (s0 + i) + 1];
            ptsn[s0 + i] = make_double4(sc1 * x1 + pi.T1[1], sc1 * y1 + pi.T1[2], sc2 * x2 + pi.T2[1],
                                        sc2 * y2 + pi.T2[2]);
            ptsr[s0 + i] = make_double4(x1, y1, x2, y2);
        }
    }
    if (threadIdx.x == 0) info[p] = pi;
}

// F in pixel space from the normalised-space solution: F = T2^T Fn T1
RS_HD void denorm_F(const double* Fn, const double* T1, const double* T2, double* F) {
    const double A[9] = {T1[0], 0, T1[1], 0, T1[0], T1[2], 0, 0, 1};
    const double B[9] = {T2[0], 0, T2[1], 0, T2[0], T2[2], 0, 0, 1};
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[i * 3 + j] = Fn[i * 3 + 0] * A[0 * 3 + j] + Fn[i * 3 + 1] * A[1 * 3 + j] + Fn[i * 3 + 2] * A[2 * 3 + j];
    double nrm = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            F[i * 3 + j] = B[0 * 3 + i] * t[0 * 3 + j] + B[1 * 3 + i] * t[1 * 3 + j] + B[2 * 3 + i] * t[2 * 3 + j];
            nrm += F[i * 3 + j] * F[i * 3 + j];
        }
    nrm = 1.0 / sqrt(nrm);
    for (int k = 0; k < 9; ++k) F[k] *= nrm;
}

// ------------------------------------------------------------------ 5-point solver, one hypothesis per 16 lanes
// The Stewenius / Nister formulation OpenCV's EMEstimatorCallback::runKernel uses
// (calib3d/five-point.cpp): the 10 cubic constraints over the 4-dim null space
// E = x X + y Y + z Z + W form a 10 x 20 coefficient matrix over the monomials
//   pivots  x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x yz^2 yz y z^3 z^2 z 1
// reduced to [I | A] by Gauss-Jordan; the pivot pairs (x^2z, x^2), (y^2z, y^2),
// (xyz, xy) give a 3 x 3 matrix of polynomials in z acting on (x, y, 1) whose
// determinant is the degree-10 polynomial; each real root z gives (x, y) from the
// matrix's null vector.  Data layout on the GPU: a 16-lane group per hypothesis (4
// per wave), the null space in LDS, constraint row r of the matrix in lane r's
// registers (20 doubles), Gauss-Jordan by cross-lane shuffles of the pivot row --
// instead of one lane carrying every intermediate (the single-lane solver above
// needed 11 KB of scratch per lane).

// column of monomial x^a y^b z^c (a + b + c <= 3) in the order above
constexpr int mono_col(int a, int b, int c) {
    return (a == 3) ? 0 : (b == 3) ? 1 : (a == 2 && b == 1) ? 2 : (a == 1 && b == 2) ? 3
         : (a == 2 && c == 1) ? 4 : (a == 2) ? 5 : (b == 2 && c == 1) ? 6 : (b == 2) ? 7
         : (a == 1 && b == 1 && c == 1) ? 8 : (a == 1 && b == 1) ? 9 : (a == 1 && c == 2) ? 10
         : (a == 1 && c == 1) ? 11 : (a == 1) ? 12 : (b == 1 && c == 2) ? 13 : (b == 1 && c == 1) ? 14
         : (b == 1) ? 15 : (c == 3) ? 16 : (c == 2) ? 17 : (c == 1) ? 18 : 19;
}
// quadratic monomials (a + b + c <= 2): index a..c -> 0..9
constexpr int QA[10] = {2, 1, 1, 1, 0, 0, 0, 0, 0, 0};
constexpr int QB[10] = {0, 1, 0, 0, 2, 1, 1, 0, 0, 0};
constexpr int QC[10] = {0, 0, 1, 0, 0, 1, 0, 2, 1, 0};
constexpr int LA[4] = {1, 0, 0, 0}, LB[4] = {0, 1, 0, 0}, LC[4] = {0, 0, 1, 0};  // x, y, z, 1
constexpr int qidx(int a, int b, int c) {
    return (a == 2) ? 0 : (a == 1 && b == 1) ? 1 : (a == 1 && c == 1) ? 2 : (a == 1) ? 3 : (b == 2) ? 4
         : (b == 1 && c == 1) ? 5 : (b == 1) ? 6 : (c == 2) ? 7 : (c == 1) ? 8 : 9;
}

// q (+)= s * (l1 * l2), linear polys l = [x, y, z, 1] coefficients
__device__ __forceinline__ void q_fma(double (&q)[10], const double* l1, const double* l2, double s) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) q[qidx(LA[i] + LA[j], LB[i] + LB[j], LC[i] + LC[j])] += s * l1[i] * l2[j];
}
// c (+)= q * l
__device__ __forceinline__ void c_fma(double (&c)[20], const double (&q)[10], const double* l) {
#pragma unroll
    for (int i = 0; i < 10; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[mono_col(QA[i] + LA[j], QB[i] + LB[j], QC[i] + LC[j])] += q[i] * l[j];
}

template <int NA, int NB>
__device__ __forceinline__ void pmul_acc(double* out, const double* a, const double* b, double s) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) out[i + j] += s * a[i] * b[j];
}

// Null space of the 5 x 9 epipolar design matrix by Householder QR of its transpose
// (9 x 5): the last 4 columns of Q = H0 H1 ... H4 are an orthonormal basis.  Fixed loop
// structure, every index static, so everything stays in registers (a pivoting
// elimination's data-dependent row / column indices put the arrays in scratch).
// Rank < 5 (a Householder diagonal below 1e-12 of the column scale) -> false.
__device__ __forceinline__ bool null_space5_reg(const double (&A)[5][9], double (&N)[4][9]) {
    double M[9][5], V[5][9], beta[5];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < 5; ++k) M[i][k] = A[k][i];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        double nrm2 = 0.0, scale = 0.0;
#pragma unroll
        for (int i = k; i < 9; ++i) nrm2 += M[i][k] * M[i][k];
#pragma unroll
        for (int i = 0; i < 9; ++i) scale += M[i][k] * M[i][k];
        const double nrm = sqrt(nrm2);
        ok = ok && nrm > 1e-12 * sqrt(scale) && nrm > 0.0;
        const double alpha = M[k][k] > 0.0 ? -nrm : nrm;
        double vn2 = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            V[k][i] = i < k ? 0.0 : (i == k ? M[k][k] - alpha : M[i][k]);
            vn2 += V[k][i] * V[k][i];
        }
        beta[k] = vn2 > 0.0 ? 2.0 / vn2 : 0.0;
#pragma unroll
        for (int j = k + 1; j < 5; ++j) {
            double s = 0.0;
#pragma unroll
            for (int i = k; i < 9; ++i) s += V[k][i] * M[i][j];
            s *= beta[k];
#pragma unroll
            for (int i = k; i < 9; ++i) M[i][j] -= s * V[k][i];
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double e[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) e[i] = (i == 5 + j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 4; k >= 0; --k) {
            double s = 0.0;
#pragma unroll
            for (int i = k; i < 9; ++i) s += V[k][i] * e[i];
            s *= beta[k];
#pragma unroll
            for (int i = k; i < 9; ++i) e[i] -= s * V[k][i];
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) N[j][i] = e[i];
    }
    return ok;
}

// Real roots of sum c[i] x^i (degree <= 10) for a 16-lane group: all roots at once by
// Aberth-Ehrlich iteration, lane i refining estimate z_i (complex) with the others'
// estimates gathered by shuffles (cubic convergence, no brackets -- OpenCV's
// solvePoly is the related Durand-Kerner iteration); estimates with a negligible
// imaginary part are the real roots, polished by two real Newton steps and
// gathered in lane order, so every lane of the group holds the same list.
// MLG_RS_ROOTS_LDS: each iteration gathers the group's estimates through LDS (one
// ds_write_b128 of (re, im) per lane, ten broadcast ds_read_b128) instead of twenty
// 64-bit shuffles (forty ds_bpermute); the same values, so the same roots.
#ifndef MLG_RS_ROOTS_LDS
#define MLG_RS_ROOTS_LDS 1
#endif
__device__ int real_roots10(double (&c)[11], double (&roots)[10], int r, int gl, double2* __restrict__ zs) {
    double mx = 0.0;
#pragma unroll
    for (int i = 0; i <= 10; ++i) mx = fmax(mx, fabs(c[i]));
    if (mx == 0.0) return 0;
    int n = 0;  // degree after dropping negligible leading coefficients
#pragma unroll
    for (int i = 1; i <= 10; ++i)
        if (fabs(c[i]) > 1e-13 * mx) n = i;
    if (n == 0) return 0;
    double lead = 0.0;
#pragma unroll
    for (int i = 1; i <= 10; ++i) lead = (i == n) ? c[i] : lead;
#pragma unroll
    for (int i = 0; i <= 10; ++i) c[i] = i <= n ? c[i] / lead : 0.0;
    // start on a circle of the roots' geometric-mean modulus |c0|^(1/n), at angles
    // 2 pi r / n + 0.4 (rs_math.h: the twin's start points, bit for bit)
    const double R = fmax(rs_root(fabs(c[0]), n), 1e-6);
    const int rr = r < 10 ? r : 9;  // 16-lane groups: lanes 10..15 hold no root
    double zr = R * RS_START_RE[n - 1][rr], zi = R * RS_START_IM[n - 1][rr];
    bool done = r >= n;
    for (int it = 0; it < 60; ++it) {
        // every lane of the group takes part in the gathers (converged ones included)
        double xr_[10], xi_[10];
        if (MLG_RS_ROOTS_LDS) {
            zs[r] = make_double2(zr, zi);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                const double2 z = zs[j];
                xr_[j] = z.x;
                xi_[j] = z.y;
            }
            __builtin_amdgcn_wave_barrier();  // reads done before the next iteration's write
        } else {
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                xr_[j] = __shfl(zr, gl + j, 64);
                xi_[j] = __shfl(zi, gl + j, 64);
            }
        }
        if (!done) {
            // p(z), p'(z) by Horner (complex), the complex products as explicit fma chains
            // (the C twin spells the same ones: this file builds without contraction)
            double pr = 0.0, pi_ = 0.0, dr = 0.0, di = 0.0;
#pragma unroll
            for (int i = 10; i >= 0; --i) {
                if (i <= n) {
                    const double ndr = fma(dr, zr, fma(-di, zi, pr)), ndi = fma(dr, zi, fma(di, zr, pi_));
                    dr = ndr; di = ndi;
                    const double npr = fma(pr, zr, fma(-pi_, zi, c[i])), npi = fma(pr, zi, pi_ * zr);
                    pr = npr; pi_ = npi;
                }
            }
            // w = p / p'
            const double dd = dr * dr + di * di;
            double wr, wi;
            if (dd > 0.0) {
                wr = (pr * dr + pi_ * di) / dd;
                wi = (pi_ * dr - pr * di) / dd;
            } else {
                wr = 1e-3 * R; wi = 1e-3 * R;  // stationary point: nudge
            }
            // s = sum_{j != i} 1 / (z_i - z_j) as one fraction num / den
            double nr_ = 0.0, ni_ = 0.0, er = 1.0, ei = 0.0;
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                if (j != r && j < n) {
                    const double ar = zr - xr_[j], ai = zi - xi_[j];
                    const double tr = fma(nr_, ar, fma(-ni_, ai, er)), ti = fma(nr_, ai, fma(ni_, ar, ei));
                    nr_ = tr; ni_ = ti;
                    const double ur = fma(er, ar, -(ei * ai)), ui = fma(er, ai, ei * ar);
                    er = ur; ei = ui;
                }
            }
            // denominator 1 - w s = (den - w num) / den;  step = w den / (den - w num)
            const double qr = er - (wr * nr_ - wi * ni_), qi = ei - (wr * ni_ + wi * nr_);
            const double mr = wr * er - wi * ei, mi = wr * ei + wi * er;
            const double qq = qr * qr + qi * qi;
            double sr = wr, si = wi;
            if (qq > 0.0 && isfinite(qq)) {
                sr = (mr * qr + mi * qi) / qq;
                si = (mi * qr - mr * qi) / qq;
            }
            zr -= sr;
            zi -= si;
            done = sr * sr + si * si <= 1e-30 * (zr * zr + zi * zi) + 1e-300;
        }
        if (__all(done)) break;
    }
    // real roots: negligible imaginary part; polish on the real polynomial
    bool real = r < n && fabs(zi) <= 1e-7 * fmax(1.0, fabs(zr));
    double x = zr;
    if (real) {
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            double f = 0.0, df = 0.0;
#pragma unroll
            for (int i = 10; i >= 0; --i)
                if (i <= n) { df = df * x + f; f = f * x + c[i]; }
            if (df != 0.0) {
                const double xn = x - f / df;
                if (isfinite(xn)) x = xn;
            }
        }
    }
    int nn = 0;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const double v = __shfl(x, gl + j, 64);
        const int isr = __shfl((int)real, gl + j, 64);
        if (isr) {
#pragma unroll
            for (int i = 0; i < 10; ++i)
                if (i == nn) roots[i] = v;
            ++nn;
        }
    }
    return nn;
}

// The 5-point sample's null space (Householder QR) one hypothesis per lane, ahead of
// k_ransac_hyp5 (MLG_RS_NULL_SPLIT): inside hyp5's 16-lane groups all 16 lanes ran the
// same QR, 4 hypotheses per wave.  The basis (36 doubles) and the rank flag (slot 36)
// go to the hypothesis' own model slot, which hyp5 reads before it writes the models.
#ifndef MLG_RS_NULL_SPLIT
#define MLG_RS_NULL_SPLIT 1
#endif
__device__ __forceinline__ bool hyp5_active(const PairInfo& pi, int h, int H, const int32_t* __restrict__ nsub, int p) {
    return h < H && (pi.mode == 5 ? h == 0 : h < nsub[p]);
}

__device__ __forceinline__ bool hyp5_null(const PairInfo& pi, const double4* __restrict__ ptsn,
                                          const int32_t* __restrict__ subsets, int p, int H, int h,
                                          double (&Nb)[4][9]) {
    double q1[5][2], q2[5][2];
    for (int i = 0; i < 5; ++i) {
        const int id = pi.mode == 5 ? i : subsets[((size_t)p * H + h) * 7 + i];
        const double4 q = ptsn[pi.start + id];
        q1[i][0] = q.x; q1[i][1] = q.y; q2[i][0] = q.z; q2[i][1] = q.w;
    }
    double A[5][9];
    for (int i = 0; i < 5; ++i) {
        const double x1 = q1[i][0], y1 = q1[i][1], x2 = q2[i][0], y2 = q2[i][1];
        A[i][0] = x2 * x1; A[i][1] = x2 * y1; A[i][2] = x2;
        A[i][3] = y2 * x1; A[i][4] = y2 * y1; A[i][5] = y2;
        A[i][6] = x1;      A[i][7] = y1;      A[i][8] = 1.0;
    }
    return null_space5_reg(A, Nb);
}

__global__ __launch_bounds__(64) void k_ransac_null5(const PairInfo* __restrict__ info, const double4* __restrict__ ptsn,
                                                     int H, const int32_t* __restrict__ subsets,
                                                     const int32_t* __restrict__ nsub, double* __restrict__ models,
                                                     int h0, int hn, const uint8_t* __restrict__ done) {
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * 64 + threadIdx.x;
    if (h >= h0 + hn || (done && done[p])) return;
    const PairInfo pi = info[p];
    if (!(pi.mode == 1 || pi.mode == 5) || !hyp5_active(pi, h, H, nsub, p)) return;
    double Nb[4][9];
    const bool ok = hyp5_null(pi, ptsn, subsets, p, H, h, Nb);
    double* o = models + ((size_t)p * H + h) * MAXSOL * 9;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int k = 0; k < 9; ++k) o[9 * a + k] = Nb[a][k];
    o[36] = ok ? 1.0 : 0.0;
}

// GS lanes per hypothesis group: 16 (4 groups per wave) or 10 (MLG_RS_G10: 6 groups, lanes
// 60..63 idle) -- the solver's ten constraint rows and ten root estimates each fill one
// lane, so 10-lane groups put 6 hypotheses on a wave instead of 4.  Same arithmetic per
// lane; the pivot search (max |a|, ties to the lowest lane) scans the group's lanes in
// order instead of an xor tree -- the same pivot for every non-NaN column.
#ifndef MLG_RS_G10
#define MLG_RS_G10 1
#endif
constexpr int HYP5_GS = MLG_RS_G10 ? 10 : 16, HYP5_GPB = 4 * (64 / HYP5_GS);  // lanes per group, groups per block
// MLG_RS_ROOTS_SPLIT: k_ransac_hyp5 stops at the degree-10 polynomial and leaves it, with
// the 3 x 3 polynomial matrix, in the hypothesis' model slot; k_ransac_roots5 then finds
// the roots and writes the models with a third of the solver's registers, so more waves
// hide the f64 latency of the root iteration.  Needs MLG_RS_NULL_SPLIT (the slot then
// holds: [0, 36) null space, [36] stage flag, [37, 48) polynomial, [48, 87) matrix).
#ifndef MLG_RS_ROOTS_SPLIT
#define MLG_RS_ROOTS_SPLIT 1
#endif
constexpr bool HYP5_ROOTS_SPLIT = MLG_RS_ROOTS_SPLIT && MLG_RS_NULL_SPLIT;
constexpr int SLOT_FLAG = 36, SLOT_POLY = 37, SLOT_MAT = 48;
constexpr double FLAG_POLY = 2.0;  // the slot's polynomial and matrix are written

// the models of one hypothesis from its real roots z (lane 0 of the group): the null
// vector of the 3 x 3 matrix at z gives (x, y); E = x X + y Y + z Z + W, normalised
// bx(i, d), by(i, d), b1(i, d): the matrix's polynomial entries; nb(a, k): the null space
template <class BX, class BY, class B1, class NB>
__device__ __forceinline__ int hyp5_models(const double (&zr)[10], int nz, BX bx, BY by, B1 b1, NB nb,
                                           double* __restrict__ out) {
    int ns = 0;
#pragma unroll
    for (int t = 0; t < 10; ++t) {
        if (t >= nz) continue;
        const double z = zr[t];
        double M[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double vx = 0.0, vy = 0.0, v1 = 0.0;
#pragma unroll
            for (int d = 3; d >= 0; --d) { vx = vx * z + bx(i, d); vy = vy * z + by(i, d); }
#pragma unroll
            for (int d = 4; d >= 0; --d) v1 = v1 * z + b1(i, d);
            M[i][0] = vx; M[i][1] = vy; M[i][2] = v1;
        }
        // null vector of the rank-2 M: the largest cross product of two rows
        double best[3] = {0.0, 0.0, 0.0}, bn = -1.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const int b = (a + 1) % 3;
            const double cx = M[a][1] * M[b][2] - M[a][2] * M[b][1];
            const double cy = M[a][2] * M[b][0] - M[a][0] * M[b][2];
            const double cz = M[a][0] * M[b][1] - M[a][1] * M[b][0];
            const double n2 = cx * cx + cy * cy + cz * cz;
            if (n2 > bn) { bn = n2; best[0] = cx; best[1] = cy; best[2] = cz; }
        }
        if (!(fabs(best[2]) > 1e-300 * sqrt(fmax(bn, 1e-300)))) continue;
        const double x = best[0] / best[2], y = best[1] / best[2];
        if (!(fabs(x) < 1e300) || !(fabs(y) < 1e300)) continue;
        double e[9], nrm = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            e[k] = x * nb(0, k) + y * nb(1, k) + z * nb(2, k) + nb(3, k);
            nrm += e[k] * e[k];
        }
        nrm = 1.0 / sqrt(nrm);
        double* Eo = out + ns * 9;
#pragma unroll
        for (int k = 0; k < 9; ++k) Eo[k] = e[k] * nrm;
        ++ns;
    }
    return ns;
}

template <int GS, bool SPLIT>
__global__ __launch_bounds__(256) void k_ransac_hyp5(const PairInfo* __restrict__ info,
                                                     const double4* __restrict__ ptsn, int H,
                                                     const int32_t* __restrict__ subsets,
                                                     const int32_t* __restrict__ nsub, double* __restrict__ models,
                                                     int8_t* __restrict__ nsol, int h0,
                                                     const uint8_t* __restrict__ done) {
    constexpr int GPW = 64 / GS, GPB = 4 * GPW;
    __shared__ double snb[GPB][4][9];
    __shared__ double2 szs[GPB][17];  // root estimates per group (17: groups on distinct banks)
    const int lane = threadIdx.x & 63, gw = lane / GS;
    const bool valid = gw < GPW;  // GS = 10: lanes 60..63 belong to no group
    const int g = (threadIdx.x >> 6) * GPW + (valid ? gw : 0), r = lane - gw * GS, gl = gw * GS;  // group, lane in group, base
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * GPB + g;
    if (done && done[p]) return;  // uniform per block
    const PairInfo pi = info[p];
    const bool ess = pi.mode == 1 || pi.mode == 5;
    // whole groups are active or not (shuffles stay inside a group)
    const bool act = valid && ess && hyp5_active(pi, h, H, nsub, p);
    if (!ess) return;  // uniform per block (one pair per blockIdx.y)
    bool ok = act;
    if (act) {
        if (MLG_RS_NULL_SPLIT) {  // k_ransac_null5 left the basis in this hypothesis' model slot
            const double* nb = models + ((size_t)p * H + h) * MAXSOL * 9;
            for (int i = r; i < 36; i += GS) snb[g][i / 9][i % 9] = nb[i];
            ok = nb[36] != 0.0;
        } else {
            double Nb[4][9];
            ok = hyp5_null(pi, ptsn, subsets, p, H, h, Nb);
            if (r == 0)
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int k = 0; k < 9; ++k) snb[g][a][k] = Nb[a][k];
        }
    }
    __syncthreads();
    if (!valid) return;  // after the barrier: no group reads these lanes
#if defined(RS_ABLATE) && RS_ABLATE == 3
    if (act && r == 0) nsol[(size_t)p * H + h] = 0;
    return;
#endif
    // E_k = [x, y, z, 1] coefficients of entry k
    auto ent = [&](int k, double* l) {
        for (int a = 0; a < 4; ++a) l[a] = snb[g][a][k];
    };
    // constraint row r (lanes 0..9): det(E) or (E E^T - tr(E E^T) / 2) E, entry (i, j)
    double row[20];
#pragma unroll
    for (int j = 0; j < 20; ++j) row[j] = 0.0;
    if (ok && r == 0) {
        const int cof[3][5] = {{0, 4, 8, 5, 7}, {1, 3, 8, 5, 6}, {2, 3, 7, 4, 6}};
        const double sg[3] = {1.0, -1.0, 1.0};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            double l0[4], l1[4], l2[4], l3[4], l4[4];
            ent(cof[t][0], l0); ent(cof[t][1], l1); ent(cof[t][2], l2); ent(cof[t][3], l3); ent(cof[t][4], l4);
            double q[10];
#pragma unroll
            for (int s = 0; s < 10; ++s) q[s] = 0.0;
            q_fma(q, l1, l2, sg[t]);
            q_fma(q, l3, l4, -sg[t]);
            c_fma(row, q, l0);
        }
    } else if (ok && r < 10) {
        const int i = (r - 1) / 3, j = (r - 1) % 3;
        double tr[10], eet[3][10];
#pragma unroll
        for (int s = 0; s < 10; ++s) {
            tr[s] = 0.0;
            eet[0][s] = 0.0; eet[1][s] = 0.0; eet[2][s] = 0.0;
        }
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            double a[4], b[4];
            for (int kk = 0; kk < 3; ++kk) {
                ent(l * 3 + kk, a);
                q_fma(tr, a, a, 0.5);
            }
            for (int kk = 0; kk < 3; ++kk) {
                ent(i * 3 + kk, a);
                ent(l * 3 + kk, b);
                q_fma(eet[l], a, b, 1.0);
            }
        }
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            double m[10];
#pragma unroll
            for (int s = 0; s < 10; ++s) m[s] = eet[l][s] - (l == i ? tr[s] : 0.0);
            double e[4];
            ent(l * 3 + j, e);
            c_fma(row, m, e);
        }
    }
    // Gauss-Jordan over the group's rows (lanes 0..9), partial pivoting; the row with
    // pivot column c ends in lane piv[c], scaled to 1 at c and 0 at the other pivots
    int piv[10];
    bool used = r >= 10;
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        double best = used ? -1.0 : fabs(row[c]);
        int bl = r;
        if constexpr (GS == 16) {
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o, 64);
                const int ol = __shfl_xor(bl, o, 64);
                if (ob > best || (ob == best && ol < bl)) { best = ob; bl = ol; }
            }
        } else {
            const double mine = best;
            best = -2.0;
            bl = GS;
#pragma unroll
            for (int jl = 0; jl < GS; ++jl) {
                const double ob = __shfl(mine, gl + jl, 64);
                if (ob > best) { best = ob; bl = jl; }
            }
        }
        if (!(best > 1e-300)) ok = false;  // singular (uniform in the group)
        piv[c] = bl;
        double prow[20];
#pragma unroll
        for (int jj = c; jj < 20; ++jj) prow[jj] = __shfl(row[jj], gl + bl, 64);
        const double inv = ok ? 1.0 / prow[c] : 0.0;
        if (r == bl) {
#pragma unroll
            for (int jj = c; jj < 20; ++jj) row[jj] = prow[jj] * inv;
            used = true;
        } else {
            const double f = row[c] * inv;
#pragma unroll
            for (int jj = c; jj < 20; ++jj) row[jj] -= f * prow[jj];
        }
    }
    // the 3 x 3 polynomial matrix on (x, y, 1) from the pivot pairs (x^2z, x^2), (y^2z, y^2),
    // (xyz, xy): column k of A = row[10 + k] of the pivot's lane
    double bx[3][4], by[3][4], b1[3][5];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double a4[10], a5[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            a4[k] = __shfl(row[10 + k], gl + piv[4 + 2 * i], 64);
            a5[k] = __shfl(row[10 + k], gl + piv[5 + 2 * i], 64);
        }
        // non-pivot columns: 0 xz^2, 1 xz, 2 x, 3 yz^2, 4 yz, 5 y, 6 z^3, 7 z^2, 8 z, 9 1
        bx[i][0] = a4[2]; bx[i][1] = a4[1] - a5[2]; bx[i][2] = a4[0] - a5[1]; bx[i][3] = -a5[0];
        by[i][0] = a4[5]; by[i][1] = a4[4] - a5[5]; by[i][2] = a4[3] - a5[4]; by[i][3] = -a5[3];
        b1[i][0] = a4[9]; b1[i][1] = a4[8] - a5[9]; b1[i][2] = a4[7] - a5[8]; b1[i][3] = a4[6] - a5[7];
        b1[i][4] = -a5[6];
    }
    if (!ok) {
        // inactive hypotheses too (5-point direct pairs beyond h = 0, RANSAC pairs beyond
        // nsub): k_ransac_score and the argmax in k_ransac_select read every slot h < H
        if (h < H && r == 0) nsol[(size_t)p * H + h] = 0;
        return;
    }
#if defined(RS_ABLATE) && RS_ABLATE == 2
    if (r == 0) nsol[(size_t)p * H + h] = (int8_t)(bx[0][0] > 1e300);
    return;
#endif
    // det = bx0 (by1 b12 - b11 by2) - by0 (bx1 b12 - b11 bx2) + b10 (bx1 by2 - by1 bx2)
    double poly[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) poly[i] = 0.0;
    {
        double t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = 0.0;
        pmul_acc<4, 5>(t, by[1], b1[2], 1.0);
        pmul_acc<5, 4>(t, b1[1], by[2], -1.0);
        pmul_acc<4, 8>(poly, bx[0], t, 1.0);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = 0.0;
        pmul_acc<4, 5>(t, bx[1], b1[2], 1.0);
        pmul_acc<5, 4>(t, b1[1], bx[2], -1.0);
        pmul_acc<4, 8>(poly, by[0], t, -1.0);
        double u[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) u[i] = 0.0;
        pmul_acc<4, 4>(u, bx[1], by[2], 1.0);
        pmul_acc<4, 4>(u, by[1], bx[2], -1.0);
        pmul_acc<5, 7>(poly, b1[0], u, 1.0);
    }
    double zr[10];
#if defined(RS_ABLATE) && RS_ABLATE == 1
    if (r == 0) nsol[(size_t)p * H + h] = (int8_t)(poly[3] > 1e300);
    return;
#endif
    if constexpr (SPLIT) {  // k_ransac_roots5 continues from the slot
        if (r == 0) {
            double* o = models + ((size_t)p * H + h) * MAXSOL * 9;
#pragma unroll
            for (int i = 0; i < 11; ++i) o[SLOT_POLY + i] = poly[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    o[SLOT_MAT + 13 * i + d] = bx[i][d];
                    o[SLOT_MAT + 13 * i + 4 + d] = by[i][d];
                }
#pragma unroll
                for (int d = 0; d < 5; ++d) o[SLOT_MAT + 13 * i + 8 + d] = b1[i][d];
            }
            o[SLOT_FLAG] = FLAG_POLY;
        }
        return;
    } else {
        const int nz = real_roots10(poly, zr, r, gl, szs[g]);
        if (r != 0) return;
        nsol[(size_t)p * H + h] = (int8_t)hyp5_models(
            zr, nz, [&](int i, int d) { return bx[i][d]; }, [&](int i, int d) { return by[i][d]; },
            [&](int i, int d) { return b1[i][d]; }, [&](int a, int k) { return snb[g][a][k]; },
            models + ((size_t)p * H + h) * MAXSOL * 9);
    }
}

// The roots and models of the hypotheses k_ransac_hyp5<.., true> left at the polynomial
// stage (same group layout; every other slot is left as it is).
template <int GS>
__global__ __launch_bounds__(256) void k_ransac_roots5(const PairInfo* __restrict__ info, int H,
                                                       const int32_t* __restrict__ nsub, double* __restrict__ models,
                                                       int8_t* __restrict__ nsol, int h0,
                                                       const uint8_t* __restrict__ done) {
    constexpr int GPW = 64 / GS, GPB = 4 * GPW;
    __shared__ double2 szs[GPB][17];
    __shared__ double scoef[GPB][39 + 36];  // the slot's matrix and null space, read before models overwrite it
    const int lane = threadIdx.x & 63, gw = lane / GS;
    const bool valid = gw < GPW;
    const int g = (threadIdx.x >> 6) * GPW + (valid ? gw : 0), r = lane - gw * GS, gl = gw * GS;
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * GPB + g;
    if (done && done[p]) return;
    const PairInfo pi = info[p];
    if (!(pi.mode == 1 || pi.mode == 5) || !valid || !hyp5_active(pi, h, H, nsub, p)) return;
    double* o = models + ((size_t)p * H + h) * MAXSOL * 9;
    if (o[SLOT_FLAG] != FLAG_POLY) return;  // group-uniform: singular sample, nsol already 0
    double* sc = scoef[g];
    for (int i = r; i < 39; i += GS) sc[i] = o[SLOT_MAT + i];
    for (int i = r; i < 36; i += GS) sc[39 + i] = o[i];
    double poly[11], zr[10];
#pragma unroll
    for (int i = 0; i < 11; ++i) poly[i] = o[SLOT_POLY + i];
    const int nz = real_roots10(poly, zr, r, gl, szs[g]);  // its LDS waits order the copies above
    if (r != 0) return;
    __builtin_amdgcn_wave_barrier();
    nsol[(size_t)p * H + h] = (int8_t)hyp5_models(
        zr, nz, [&](int i, int d) { return sc[13 * i + d]; }, [&](int i, int d) { return sc[13 * i + 4 + d]; },
        [&](int i, int d) { return sc[13 * i + 8 + d]; }, [&](int a, int k) { return sc[39 + 9 * a + k]; }, o);
}

// OpenCV's sample stream for pair p (modes 1 / 2): subsets of iterations 0..nsub-1.
// getSubset: draw modelPoints indices with cv::RNG, redrawing duplicates; for F the
// whole subset is redrawn while checkSubset (collinear points in either image) fails,
// up to 10000 attempts; an iteration whose getSubset fails ends the loop.
__global__ __launch_bounds__(64) void k_ransac_subsets(const PairInfo* __restrict__ info, int P, int H,
                                                       const float* __restrict__ kp1, const float* __restrict__ kp2,
                                                       int32_t* __restrict__ subsets, int32_t* __restrict__ nsub) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const PairInfo pi = info[p];
    if (pi.mode != 1 && pi.mode != 2) {
        nsub[p] = 0;
        return;
    }
    const int m = pi.mode == 1 ? 5 : 7;
    CvRng rng{~0ull};
    int32_t* out = subsets + (size_t)p * H * 7;
    int it = 0;
    for (; it < H; ++it) {
        int idx[7];
        float a[7][2], b[7][2];
        int iters = 0, i = 0;
        for (; iters < RANSAC_MAX_ATTEMPTS; ++iters) {
            for (i = 0; i < m;) {
                int v;
                for (;;) {
                    v = idx[i] = rng.uniform(0, pi.count);
                    int j = 0;
                    for (; j < i; ++j)
                        if (v == idx[j]) break;
                    if (j == i) break;
                }
                a[i][0] = kp1[2 * (pi.start + v)]; a[i][1] = kp1[2 * (pi.start + v) + 1];
                b[i][0] = kp2[2 * (pi.start + v)]; b[i][1] = kp2[2 * (pi.start + v) + 1];
                ++i;
            }
            if (m == 7 && (collinear_last(a, 7) || collinear_last(b, 7))) continue;
            break;
        }
        if (!(i == m && iters < RANSAC_MAX_ATTEMPTS)) break;
        for (int j = 0; j < m; ++j) out[it * 7 + j] = idx[j];
    }
    nsub[p] = it;
}

__global__ __launch_bounds__(64) void k_ransac_hyp(const PairInfo* __restrict__ info, const double4* __restrict__ ptsn,
                                                   int H, uint64_t seed, const int32_t* __restrict__ subsets,
                                                   const int32_t* __restrict__ nsub, double* __restrict__ models,
                                                   int8_t* __restrict__ nsol, int h0, const uint8_t* __restrict__ done) {
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H || (done && done[p])) return;
    const PairInfo pi = info[p];
    double* out = models + ((size_t)p * H + h) * MAXSOL * 9;
    if (pi.mode == 1 || pi.mode == 5) return;  // essential matrix: k_ransac_null5 / hyp5 / roots5
    const bool direct = pi.mode == 4;          // 7 points: the 7-point models directly
    if (pi.mode == 0 || (direct && h > 0)) {
        nsol[(size_t)p * H + h] = 0;
        return;
    }
    int idx[7];
    if (direct) {
        for (int i = 0; i < 7; ++i) idx[i] = i;
    } else if (pi.mode == 2) {  // RANSAC: OpenCV's sample stream (k_ransac_subsets)
        if (h >= nsub[p]) {
            nsol[(size_t)p * H + h] = 0;
            return;
        }
        for (int i = 0; i < 7; ++i) idx[i] = subsets[((size_t)p * H + h) * 7 + i];
    } else {  // LMedS: the stream depends on (seed, h) only, so a pair's result does not depend on the batch
        uint64_t st = splitmix(seed ^ (uint64_t)h * 0x632BE59BD9B4E019ull);
        for (int i = 0; i < 7; ++i) {
            int v;
            bool dup;
            do {
                st = splitmix(st);
                v = (int)((st >> 11) % (uint64_t)pi.count);
                dup = false;
                for (int j = 0; j < i; ++j) dup |= idx[j] == v;
            } while (dup);
            idx[i] = v;
        }
    }
    double q1[7][2], q2[7][2];
    for (int i = 0; i < 7; ++i) {
        const double4 q = ptsn[pi.start + idx[i]];
        q1[i][0] = q.x; q1[i][1] = q.y; q2[i][0] = q.z; q2[i][1] = q.w;
    }
    double Fn[3 * 9];
    const int ns = solve_7pt(q1, q2, Fn);
    for (int s = 0; s < ns; ++s) denorm_F(Fn + s * 9, pi.T1, pi.T2, out + s * 9);
    nsol[(size_t)p * H + h] = (int8_t)ns;
}

// score[p][h][s]: inlier count (RANSAC / direct) or -median error (LMedS); -inf if absent
__global__ __launch_bounds__(256) void k_ransac_score(const PairInfo* __restrict__ info, const double4* __restrict__ ptsn,
                                                      const double4* __restrict__ ptsr, int H,
                                                      const double* __restrict__ models,
                                                      const int8_t* __restrict__ nsol, float* __restrict__ score,
                                                      int h0, const uint8_t* __restrict__ done) {
    __shared__ double4 sp[RS_CHUNK];
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (done && done[p]) return;  // uniform per block: the barrier count stays uniform
    const PairInfo pi = info[p];
    if (pi.mode == 0) {
        if (h < H)
            for (int s = 0; s < MAXSOL; ++s) score[((size_t)p * H + h) * MAXSOL + s] = -INFINITY;
        return;
    }
    const bool ess = pi.mode == 1 || pi.mode == 5;
    const double4* src = (ess ? ptsn : ptsr) + pi.start;
    const int ns = h < H ? nsol_at(nsol, (size_t)p * H + h) : 0;
    // waves skip the loads of absent hypotheses but keep the barrier count uniform
    int cnt[MAXSOL];
    for (int s = 0; s < MAXSOL; ++s) cnt[s] = 0;
    const float t2 = (float)pi.thr2;
    // midpoint between t2 and the next float up; exactly representable in double
    const double t2_hi = 0.5 * ((double)t2 + (double)nextafterf(t2, INFINITY));
    const double* mh = models + ((size_t)p * H + (h < H ? h : 0)) * MAXSOL * 9;
    if (pi.mode == 3) {
        // LMedS: fewer than 15 points; median of the errors per model
        for (int s = 0; s < MAXSOL; ++s) {
            float med = INFINITY;
            if (s < ns) {
                float e[16];
                for (int i = 0; i < pi.count; ++i) {
                    const double4 q = src[i];
                    e[i] = err_epiline(mh + s * 9, q.x, q.y, q.z, q.w);
                }
                for (int i = 1; i < pi.count; ++i) {  // insertion sort
                    const float v = e[i];
                    int j = i - 1;
                    while (j >= 0 && e[j] > v) { e[j + 1] = e[j]; --j; }
                    e[j + 1] = v;
                }
                med = e[pi.count / 2];
            }
            if (h < H) score[((size_t)p * H + h) * MAXSOL + s] = s < ns ? -med : -INFINITY;
        }
        return;
    }
    for (int c0 = 0; c0 < pi.count; c0 += RS_CHUNK) {
        const int cn = min(RS_CHUNK, pi.count - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < cn; i += blockDim.x) sp[i] = src[c0 + i];
        __syncthreads();
        for (int s = 0; s < ns; ++s) {
            double M[9];
            for (int k = 0; k < 9; ++k) M[k] = mh[s * 9 + k];
            int c = 0;
            if (ess) {
                for (int i = 0; i < cn; ++i) {
                    const double4 q = sp[i];
                    c += sampson_inlier(M, q.x, q.y, q.z, q.w, t2, t2_hi);
                }
            } else {
                for (int i = 0; i < cn; ++i) {
                    const double4 q = sp[i];
                    c += err_epiline(M, q.x, q.y, q.z, q.w) <= t2;
                }
            }
            cnt[s] += c;
        }
    }
    if (h < H)
        for (int s = 0; s < MAXSOL; ++s)
            score[((size_t)p * H + h) * MAXSOL + s] = s < ns ? (float)cnt[s] : -INFINITY;
}

// ------------------------------------------------------------------ pose (recoverPose)
// Symmetric 3x3 eigen-decomposition (cyclic Jacobi): A = V diag(w) V^T.
RS_HD void jacobi3(double (&A)[3][3], double (&V)[3][3], double (&w)[3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
        if (off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (fabs(A[p][q]) < 1e-300) continue;
                const double th = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < 3; ++i) w[i] = A[i][i];
}

// E = U diag(s) V^T with s descending; det(U), det(V) made positive (as OpenCV's
// decomposeEssentialMat after its SVD).  Returns R1 = U W V^T, R2 = U W^T V^T, t = U[:,2].
RS_HD void decompose_E(const double* E, double (&R1)[3][3], double (&R2)[3][3], double (&t)[3]) {
    double A[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = E[0 * 3 + i] * E[0 * 3 + j] + E[1 * 3 + i] * E[1 * 3 + j] + E[2 * 3 + i] * E[2 * 3 + j];
    double V[3][3], w[3];
    jacobi3(A, V, w);
    int o[3] = {0, 1, 2};  // sort descending
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (w[o[j]] > w[o[i]]) { int tt = o[i]; o[i] = o[j]; o[j] = tt; }
    double Vs[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Vs[i][j] = V[i][o[j]];
    double U[3][3];
    for (int c = 0; c < 2; ++c) {
        double n = 0.0;
        for (int i = 0; i < 3; ++i) {
            U[i][c] = E[i * 3 + 0] * Vs[0][c] + E[i * 3 + 1] * Vs[1][c] + E[i * 3 + 2] * Vs[2][c];
            n += U[i][c] * U[i][c];
        }
        n = n > 0 ? 1.0 / sqrt(n) : 0.0;
        for (int i = 0; i < 3; ++i) U[i][c] *= n;
    }
    // u2 orthogonal to u1 (numerical hygiene), u3 = u1 x u2
    double d = U[0][0] * U[0][1] + U[1][0] * U[1][1] + U[2][0] * U[2][1];
    double n2 = 0.0;
    for (int i = 0; i < 3; ++i) { U[i][1] -= d * U[i][0]; n2 += U[i][1] * U[i][1]; }
    n2 = 1.0 / sqrt(n2);
    for (int i = 0; i < 3; ++i) U[i][1] *= n2;
    U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
    U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
    U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
    double Uc[9], Vc[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) { Uc[i * 3 + j] = U[i][j]; Vc[i * 3 + j] = Vs[i][j]; }
    if (det3(Uc) < 0)
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) U[i][j] = -U[i][j];
    if (det3(Vc) < 0)
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Vs[i][j] = -Vs[i][j];
    const double W[3][3] = {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0.0, b = 0.0;
            for (int k = 0; k < 3; ++k)
                for (int l = 0; l < 3; ++l) {
                    a += U[i][k] * W[k][l] * Vs[j][l];
                    b += U[i][k] * W[l][k] * Vs[j][l];
                }
            R1[i][j] = a;
            R2[i][j] = b;
        }
    for (int i = 0; i < 3; ++i) t[i] = U[i][2];
}

// Linear triangulation (DLT null vector via the 4x4 normal matrix) with P0 = [I|0],
// P1 = [R|t]; OpenCV's recoverPose test: z*w > 0, depth < dist in both cameras.
RS_HD bool cheiral(const double (&R)[3][3], const double (&t)[3], double x1, double y1, double x2, double y2,
                        double dist) {
    double P1[3][4];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) P1[i][j] = R[i][j];
        P1[i][3] = t[i];
    }
    const double P0[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
    double A[4][4];
    for (int j = 0; j < 4; ++j) {
        A[0][j] = x1 * P0[2][j] - P0[0][j];
        A[1][j] = y1 * P0[2][j] - P0[1][j];
        A[2][j] = x2 * P1[2][j] - P1[0][j];
        A[3][j] = y2 * P1[2][j] - P1[1][j];
    }
    // null vector of A: smallest eigenvector of A^T A by inverse iteration on a
    // Gaussian-eliminated A (4 x 4, rank 3 for exact data)
    double M[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[k][i] * A[k][j];
            M[i][j] = s;
        }
    // shift-free inverse iteration with a tiny regulariser
    double tr = M[0][0] + M[1][1] + M[2][2] + M[3][3];
    for (int i = 0; i < 4; ++i) M[i][i] += 1e-15 * tr;
    // LU of M (symmetric positive definite): Cholesky
    double L[4][4] = {{0}};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = M[i][j];
            for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
            if (i == j) {
                L[i][i] = sqrt(fmax(s, 1e-300));
            } else {
                L[i][j] = s / L[j][j];
            }
        }
    double X[4] = {0.5, 0.5, 0.5, 0.5};
    for (int it = 0; it < 6; ++it) {
        double y[4];
        for (int i = 0; i < 4; ++i) {
            double s = X[i];
            for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
            y[i] = s / L[i][i];
        }
        for (int i = 3; i >= 0; --i) {
            double s = y[i];
            for (int k = i + 1; k < 4; ++k) s -= L[k][i] * X[k];
            X[i] = s / L[i][i];
        }
        double n = sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2] + X[3] * X[3]);
        for (int i = 0; i < 4; ++i) X[i] /= n;
    }
    if (!(X[2] * X[3] > 0)) return false;
    const double X0 = X[0] / X[3], X1 = X[1] / X[3], X2 = X[2] / X[3];
    if (!(X2 < dist)) return false;
    const double z2 = R[2][0] * X0 + R[2][1] * X1 + R[2][2] * X2 + t[2];
    return z2 > 0 && z2 < dist;
}

// Adaptive early stop across two launch rounds: after hypotheses [0, H1) are solved and
// scored, replay OpenCV's sequential scan over them (as k_ransac_select does); a pair is
// done when the scan stops inside the first H1 -- its adaptive iteration budget or its
// subset count fell to <= H1 -- so the scan never reads a hypothesis >= H1 and round two
// skips the pair.  Only the sequential modes (5-point E, 7-point F) can finish early.
__global__ __launch_bounds__(256) void k_ransac_probe(const PairInfo* __restrict__ info, int P, int H, int H1,
                                                      const float* __restrict__ score,
                                                      const int8_t* __restrict__ nsol,
                                                      const int32_t* __restrict__ nsub, uint8_t* __restrict__ done) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const PairInfo pi = info[p];
    uint8_t d = 0;
    if (pi.mode == 1 || pi.mode == 2) {
        const int mp = pi.mode == 1 ? 5 : 7;
        const int ns_it = nsub[p], total = H * MAXSOL;
        int niters = H, max_good = 0;
        for (int it = 0; it < niters && it < ns_it && it < H1; ++it) {
            const int ns = nsol_at(nsol, (size_t)p * H + it);
            for (int s = 0; s < ns; ++s) {
                const int g = (int)score[(size_t)p * total + it * MAXSOL + s];
                if (g > max(max_good, mp - 1)) {
                    max_good = g;
                    niters = ransac_update_iters(RANSAC_CONFIDENCE, (double)(pi.count - g) / pi.count, mp, niters);
                }
            }
        }
        d = (niters <= H1 || ns_it <= H1) ? 1 : 0;
    }
    done[p] = d;
}

__global__ __launch_bounds__(256) void k_ransac_select(const PairInfo* __restrict__ info,
                                                       const double4* __restrict__ ptsn,
                                                       const double4* __restrict__ ptsr, int H,
                                                       const double* __restrict__ models,
                                                       const float* __restrict__ score, const int8_t* __restrict__ nsol,
                                                       const int32_t* __restrict__ nsub, double* __restrict__ model_out,
                                                       uint8_t* __restrict__ mask, int32_t* __restrict__ inliers,
                                                       int32_t* __restrict__ status) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const PairInfo pi = info[p];
    __shared__ float bs[256];
    __shared__ int bi[256];
    __shared__ double Mb[9];
    __shared__ int cnt_sh;
    const int total = H * MAXSOL;
    if (pi.mode == 1 || pi.mode == 2) {
        // OpenCV's sequential loop over iterations 0 .. niters-1 (niters shrinks as better
        // models arrive); one thread: at most H * MAXSOL comparisons
        if (tid == 0) {
            const int mp = pi.mode == 1 ? 5 : 7;
            const int ns_it = nsub[p];
            int niters = H, max_good = 0, bidx = -1;
            for (int it = 0; it < niters && it < ns_it; ++it) {
                const int ns = nsol_at(nsol, (size_t)p * H + it);
                for (int s = 0; s < ns; ++s) {
                    const int g = (int)score[(size_t)p * total + it * MAXSOL + s];
                    if (g > max(max_good, mp - 1)) {
                        max_good = g;
                        bidx = it * MAXSOL + s;
                        niters = ransac_update_iters(RANSAC_CONFIDENCE, (double)(pi.count - g) / pi.count, mp, niters);
                    }
                }
            }
            bs[0] = bidx >= 0 ? (float)max_good : -INFINITY;
            bi[0] = bidx >= 0 ? bidx : 0;
        }
        __syncthreads();
    } else {
        float best = -INFINITY;
        int bidx = 0x7fffffff;
        for (int i = tid; i < total; i += 256) {
            const float v = score[(size_t)p * total + i];
            if (v > best || (v == best && i < bidx)) { best = v; bidx = i; }
        }
        bs[tid] = best;
        bi[tid] = bidx;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (tid < o) {
                const float v = bs[tid + o];
                const int ii = bi[tid + o];
                if (v > bs[tid] || (v == bs[tid] && ii < bi[tid])) { bs[tid] = v; bi[tid] = ii; }
            }
            __syncthreads();
        }
    }
    const bool have = pi.mode != 0 && bs[0] > -INFINITY;
    if (!have) {
        for (int i = tid; i < pi.count; i += 256) mask[pi.start + i] = 0;
        if (tid == 0) {
            status[p] = 1;
            inliers[p] = 0;
            for (int k = 0; k < 9; ++k) model_out[p * 9 + k] = 0.0;
        }
        return;
    }
    if (tid < 9) Mb[tid] = models[(size_t)p * total * 9 + (size_t)bi[0] * 9 + tid];
    if (tid == 0) cnt_sh = 0;
    __syncthreads();
    const bool ess = pi.mode == 1 || pi.mode == 5;
    const bool all_in = pi.mode == 4 || pi.mode == 5;
    float t2 = (float)pi.thr2;
    if (pi.mode == 3) {  // LMedS inlier threshold from the best median
        const double med = -(double)bs[0];
        double sigma = 2.5 * 1.4826 * (1.0 + 5.0 / (pi.count - 7)) * sqrt(med);
        sigma = fmax(sigma, 0.001);
        t2 = (float)(sigma * sigma);
    }
    int c = 0;
    for (int i = tid; i < pi.count; i += 256) {
        bool in;
        if (all_in) {
            in = true;
        } else {
            const double4 q = ess ? ptsn[pi.start + i] : ptsr[pi.start + i];
            const float e = ess ? err_sampson(Mb, q.x, q.y, q.z, q.w) : err_epiline(Mb, q.x, q.y, q.z, q.w);
            in = e <= t2;
        }
        mask[pi.start + i] = in;
        c += in;
    }
    atomicAdd(&cnt_sh, c);
    __syncthreads();
    const int n_in = cnt_sh;
    if (tid == 0) {
        status[p] = 0;
        inliers[p] = n_in;
        for (int k = 0; k < 9; ++k) model_out[p * 9 + k] = Mb[k];
    }
}

// recoverPose (distanceThresh 50) of one pair per workgroup from E and the inlier
// mask; points normalised by K.  pose [P, 16]; status set to 2 when < 5 inliers.
__global__ __launch_bounds__(256) void k_recover_pose(const float* __restrict__ kp1, const float* __restrict__ kp2,
                                                      const int32_t* __restrict__ offs, const double* __restrict__ K,
                                                      int k_stride, const double* __restrict__ Es,
                                                      const uint8_t* __restrict__ mask, double* __restrict__ pose,
                                                      int32_t* __restrict__ status) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const int s0 = offs[p], S = offs[p + 1] - offs[p];
    __shared__ int good[4];
    __shared__ int nin;
    if (tid < 4) good[tid] = 0;
    if (tid == 0) nin = 0;
    __syncthreads();
    int c = 0;
    for (int i = tid; i < S; i += 256) c += mask[s0 + i] != 0;
    atomicAdd(&nin, c);
    __syncthreads();
    if (status && status[p] == 1) {
        if (tid < 16) pose[p * 16 + tid] = 0.0;
        return;
    }
    if (nin < 5) {
        if (tid < 16) pose[p * 16 + tid] = 0.0;
        if (tid == 0 && status) status[p] = 2;
        return;
    }
    const double* Kp = K + (size_t)p * k_stride;
    const double fx = Kp[0], fy = Kp[4], cx = Kp[2], cy = Kp[5];
    double E[9];
    for (int k = 0; k < 9; ++k) E[k] = Es[p * 9 + k];
    double R1[3][3], R2[3][3], tv[3];
    decompose_E(E, R1, R2, tv);
    double nt[3] = {-tv[0], -tv[1], -tv[2]};
    int g[4] = {0, 0, 0, 0};
    for (int i = tid; i < S; i += 256) {
        if (!mask[s0 + i]) continue;
        const double x1 = (kp1[2 * (s0 + i)] - cx) / fx, y1 = (kp1[2 * (s0 + i) + 1] - cy) / fy;
        const double x2 = (kp2[2 * (s0 + i)] - cx) / fx, y2 = (kp2[2 * (s0 + i) + 1] - cy) / fy;
        g[0] += cheiral(R1, tv, x1, y1, x2, y2, 50.0);
        g[1] += cheiral(R2, tv, x1, y1, x2, y2, 50.0);
        g[2] += cheiral(R1, nt, x1, y1, x2, y2, 50.0);
        g[3] += cheiral(R2, nt, x1, y1, x2, y2, 50.0);
    }
    for (int k = 0; k < 4; ++k) atomicAdd(&good[k], g[k]);
    __syncthreads();
    if (tid == 0) {
        const int a = good[0], b = good[1], cc = good[2], d = good[3];
        int pick;
        if (a >= b && a >= cc && a >= d) pick = 0;
        else if (b >= a && b >= cc && b >= d) pick = 1;
        else if (cc >= a && cc >= b && cc >= d) pick = 2;
        else pick = 3;
        const double (*R)[3] = (pick & 1) ? R2 : R1;
        const double* tt = (pick & 2) ? nt : tv;
        double* T = pose + p * 16;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i][j];
            T[i * 4 + 3] = tt[i];
        }
        T[12] = 0.0; T[13] = 0.0; T[14] = 0.0; T[15] = 1.0;
    }
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// mlg_dbg_ransac_poison_nsol: overwrite the counts of the slots no scan uses
bool g_poison_nsol = false;
int g_poison_value = 0;

__global__ __launch_bounds__(64) void k_ransac_poison_nsol(const PairInfo* __restrict__ info, int H,
                                                           const int32_t* __restrict__ nsub, int8_t* __restrict__ nsol,
                                                           int h0, int hn, const uint8_t* __restrict__ done, int value) {
    const int p = blockIdx.y;
    const int h = h0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= h0 + hn || h >= H || (done && done[p])) return;
    const int mode = info[p].mode;
    const bool unused = mode == 0 || ((mode == 4 || mode == 5) && h > 0) || ((mode == 1 || mode == 2) && h >= nsub[p]);
    if (unused) nsol[(size_t)p * H + h] = (int8_t)value;
}

struct RsLayout {
    size_t info, ptsn, ptsr, models, nsol, score, subsets, nsub, done, total;
};

RsLayout rs_layout(int P, long S_total, int H) {
    RsLayout L;
    L.info = 0;
    L.ptsn = align256(sizeof(PairInfo) * (size_t)P);
    L.ptsr = L.ptsn + align256(sizeof(double4) * (size_t)S_total);
    L.models = L.ptsr + align256(sizeof(double4) * (size_t)S_total);
    L.nsol = L.models + align256(sizeof(double) * 9 * MAXSOL * (size_t)P * H);
    L.score = L.nsol + align256((size_t)P * H);
    L.subsets = L.score + align256(sizeof(float) * MAXSOL * (size_t)P * H);
    L.nsub = L.subsets + align256(sizeof(int32_t) * 7 * (size_t)P * H);
    L.done = L.nsub + align256(sizeof(int32_t) * (size_t)P);
    L.total = L.done + align256((size_t)P);
    return L;
}

}  // namespace

size_t mlg_ransac_ws_bytes(int P, long S_total, int H) {
    if (P <= 0 || S_total < 0 || H <= 0) return 0;
    return rs_layout(P, S_total, H).total;
}

int mlg_ransac_run(const float* kp1, const float* kp2, const int32_t* offs, int P, long S_total, const double* K,
                   int k_stride, double thr, int H, uint64_t seed, void* ws, size_t ws_bytes, double* model_out,
                   uint8_t* mask, int32_t* inliers, double* pose, int32_t* status, hipStream_t s) {
    if (P <= 0 || H <= 0 || H > (1 << 20) || !(thr > 0.0) || S_total < 0) return MLG_EINVAL;
    const RsLayout L = rs_layout(P, S_total, H);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* w = (char*)ws;
    PairInfo* info = (PairInfo*)(w + L.info);
    double4* ptsn = (double4*)(w + L.ptsn);
    double4* ptsr = (double4*)(w + L.ptsr);
    double* models = (double*)(w + L.models);
    int8_t* nsol = (int8_t*)(w + L.nsol);
    float* score = (float*)(w + L.score);
    int32_t* subsets = (int32_t*)(w + L.subsets);
    int32_t* nsub = (int32_t*)(w + L.nsub);
    hipLaunchKernelGGL(k_ransac_prep, dim3(P), dim3(256), 0, s, kp1, kp2, offs, K, k_stride, thr, info, ptsn, ptsr);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_ransac_subsets, dim3((P + 63) / 64), dim3(64), 0, s, info, P, H, kp1, kp2, subsets, nsub);
    MLG_LAUNCH_CHECK();
    uint8_t* done = (uint8_t*)(w + L.done);
    // round one: hypotheses [0, H1) of every pair; round two: [H1, H) of the pairs whose
    // sequential scan has not stopped inside round one (k_ransac_probe)
    const int H1 = std::min(H, RS_ROUND1);
    for (int round = 0; round < 2; ++round) {
        const int h0 = round ? H1 : 0, hn = round ? H - H1 : H1;
        const uint8_t* skip = round ? done : nullptr;
        if (hn <= 0) break;
        hipLaunchKernelGGL(k_ransac_hyp, dim3((hn + 63) / 64, P), dim3(64), 0, s, info, ptsn, H, seed, subsets, nsub,
                           models, nsol, h0, skip);
        MLG_LAUNCH_CHECK();
        if (MLG_RS_NULL_SPLIT) {
            hipLaunchKernelGGL(k_ransac_null5, dim3((hn + 63) / 64, P), dim3(64), 0, s, info, ptsn, H, subsets, nsub,
                               models, h0, hn, skip);
            MLG_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL((k_ransac_hyp5<HYP5_GS, HYP5_ROOTS_SPLIT>), dim3((hn + HYP5_GPB - 1) / HYP5_GPB, P),
                           dim3(256), 0, s, info, ptsn, H, subsets, nsub, models, nsol, h0, skip);
        if (HYP5_ROOTS_SPLIT) {
            MLG_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_ransac_roots5<HYP5_GS>, dim3((hn + HYP5_GPB - 1) / HYP5_GPB, P), dim3(256), 0, s, info,
                               H, nsub, models, nsol, h0, skip);
        }
        MLG_LAUNCH_CHECK();
        if (g_poison_nsol) {
            hipLaunchKernelGGL(k_ransac_poison_nsol, dim3((hn + 63) / 64, P), dim3(64), 0, s, info, H, nsub, nsol, h0,
                               hn, skip, g_poison_value);
            MLG_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(k_ransac_score, dim3((hn + 255) / 256, P), dim3(256), 0, s, info, ptsn, ptsr, H, models,
                           nsol, score, h0, skip);
        MLG_LAUNCH_CHECK();
        if (round == 0 && H1 < H) {
            hipLaunchKernelGGL(k_ransac_probe, dim3((P + 255) / 256), dim3(256), 0, s, info, P, H, H1, score, nsol,
                               nsub, done);
            MLG_LAUNCH_CHECK();
        }
    }
    hipLaunchKernelGGL(k_ransac_select, dim3(P), dim3(256), 0, s, info, ptsn, ptsr, H, models, score, nsol, nsub, model_out,
                       mask, inliers, status);
    MLG_LAUNCH_CHECK();
    if (pose && K) {
        hipLaunchKernelGGL(k_recover_pose, dim3(P), dim3(256), 0, s, kp1, kp2, offs, K, k_stride, model_out, mask, pose,
                           status);
        MLG_LAUNCH_CHECK();
    }
    return MLG_OK;
}

int mlg_recover_pose_run(const float* kp1, const float* kp2, const int32_t* offs, int P, const double* K,
                         int k_stride, const double* E, const uint8_t* mask, double* pose, hipStream_t s) {
    if (P <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_recover_pose, dim3(P), dim3(256), 0, s, kp1, kp2, offs, K, k_stride, E, mask, pose,
                       (int32_t*)nullptr);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

extern "C" int mlg_dbg_ransac_poison_nsol(int on, int value) {
    g_poison_nsol = on != 0;
    g_poison_value = value;
    return MLG_OK;
}
