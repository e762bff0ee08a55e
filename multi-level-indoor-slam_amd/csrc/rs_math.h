/* Math shared by the GPU RANSAC (csrc/ransac.hip) and its C twin (oracle/csrc/ransac_cv.c).
 *
 * Every value here feeds a branch, a root or an inlier count of the epipolar RANSAC, so
 * the two sides must produce the same bits.  Library calls do not: ocml's cos / sin / pow
 * / log / hypot are not glibc's.  These are written from IEEE-exact operations only
 * (+ - * / sqrt, frexp / ldexp) and a constant table, and both sides build without FP
 * contraction, so the GPU and the twin agree bit for bit (the
 * reference's call: geometric_verification.py:128-146, OpenCV's RANSACUpdateNumIters in
 * calib3d/ptsetreg.cpp).
 *
 * The includer defines RS_FN (function qualifiers: `__host__ __device__ static inline` in
 * HIP, `static inline` in C) and RS_CONST (the table's storage: `static __constant__ const`
 * in HIP, `static const` in C) before including.  Plain C99: no C++ in here. */
#ifndef MLG_RS_MATH_H
#define MLG_RS_MATH_H

#if !defined(RS_FN) || !defined(RS_CONST)
#error "define RS_FN and RS_CONST before including rs_math.h"
#endif

/* Aberth start points: cos / sin of 2 pi r / n + 0.4 (row n - 1, column r < n; zero for
 * r >= n), exact hexadecimal doubles from tools/gen_rs_start_table.py */
RS_CONST double RS_START_RE[10][10] = {
    {0x1.d7954e7dba2f8p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, -0x1.d7954e7dba2f9p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, -0x1.98762f29e393dp-1, -0x1.f8f8fa9eb4dd0p-4, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, -0x1.8ec3ae92b6768p-2, -0x1.d7954e7dba2f9p-1, 0x1.8ec3ae92b676dp-2, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, -0x1.5f2c08503a8c7p-4, -0x1.f2b6774fec871p-1, -0x1.08532eee8b101p-1, 0x1.4f59d8cac4b97p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, 0x1.f8f8fa9eb4dc7p-4, -0x1.98762f29e393dp-1, -0x1.d7954e7dba2f9p-1, -0x1.f8f8fa9eb4dd0p-4, 0x1.98762f29e3941p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, 0x1.1449c234876c4p-2, -0x1.2b5205fefecafp-1, -0x1.ff63f7b67f490p-1, -0x1.525f849c659a7p-1, 0x1.65c8d471f3298p-3, 0x1.c1e91d9d68fe9p-1, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, 0x1.80f34d5c04145p-2, -0x1.8ec3ae92b6768p-2, -0x1.da71b6ff2c3e9p-1, -0x1.d7954e7dba2f9p-1, -0x1.80f34d5c04140p-2, 0x1.8ec3ae92b676dp-2, 0x1.da71b6ff2c3ebp-1, 0x0p+0, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, 0x1.d22fc64f27e90p-2, -0x1.c9daaf53c9048p-3, -0x1.98762f29e393dp-1, -0x1.ff56047c4a5d4p-1, -0x1.76f3578d2d114p-1, -0x1.f8f8fa9eb4dd0p-4, 0x1.163e2154b668cp-1, 0x1.e96a03621f524p-1, 0x0p+0},
    {0x1.d7954e7dba2f8p-1, 0x1.08532eee8b103p-1, -0x1.5f2c08503a8c7p-4, -0x1.4f59d8cac4b95p-1, -0x1.f2b6774fec871p-1, -0x1.d7954e7dba2f9p-1, -0x1.08532eee8b101p-1, 0x1.5f2c08503a8dep-4, 0x1.4f59d8cac4b97p-1, 0x1.f2b6774fec871p-1},
};
RS_CONST double RS_START_IM[10][10] = {
    {0x1.8ec3ae92b676bp-2, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, -0x1.8ec3ae92b6767p-2, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.34b6430d1d8a5p-1, -0x1.fc181a5678c57p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.d7954e7dba2f8p-1, -0x1.8ec3ae92b6767p-2, -0x1.d7954e7dba2f7p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.fe1d62c483ff6p-1, 0x1.cf8b5a26ac140p-3, -0x1.b67e458544eb5p-1, -0x1.82e3cb1245544p-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.fc181a5678c58p-1, 0x1.34b6430d1d8a5p-1, -0x1.8ec3ae92b6767p-2, -0x1.fc181a5678c57p-1, -0x1.34b6430d1d89fp-1, 0x0p+0, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.ed02e9a9925ecp-1, 0x1.9f6497ce8361cp-1, 0x1.8f9a344c5da38p-5, -0x1.803fdb6b32b3ep-1, -0x1.f8205967b6c73p-1, -0x1.e8c58e669ab55p-2, 0x0p+0, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.da71b6ff2c3eap-1, 0x1.d7954e7dba2f8p-1, 0x1.80f34d5c04146p-2, -0x1.8ec3ae92b6767p-2, -0x1.da71b6ff2c3ebp-1, -0x1.d7954e7dba2f7p-1, -0x1.80f34d5c04141p-2, 0x0p+0, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.c7dd0cc6218e6p-1, 0x1.f30a8a64a6b65p-1, 0x1.34b6430d1d8a5p-1, -0x1.a11279638715bp-5, -0x1.5ca620c2d2361p-1, -0x1.fc181a5678c57p-1, -0x1.adcbe52fe91cep-1, -0x1.2cc8d343a9006p-2, 0x0p+0},
    {0x1.8ec3ae92b676bp-2, 0x1.b67e458544eb3p-1, 0x1.fe1d62c483ff6p-1, 0x1.82e3cb1245546p-1, 0x1.cf8b5a26ac140p-3, -0x1.8ec3ae92b6767p-2, -0x1.b67e458544eb5p-1, -0x1.fe1d62c483ff6p-1, -0x1.82e3cb1245544p-1, -0x1.cf8b5a26ac134p-3},
};

/* x^(1/n), n = 1..10, for x >= 0 (NaN / inf / 0 returned as they are): x = m 2^e with
 * e = q n + k (0 <= k < n), so y = m 2^k lies in [0.5, 2^(n-1)) and its root in [0.5, 2);
 * Newton's step on t^n = y from t = 2 (above the root: the iterates fall monotonically)
 * until it stops falling.  The Aberth start radius only; not a correctly rounded root. */
RS_FN double rs_root(double x, int n) {
    if (!(x > 0.0) || !(x <= 1.7976931348623157e308) || n <= 1) return x;
    int e;
    const double m = frexp(x, &e);
    const int q = e >= 0 ? e / n : -((-e + n - 1) / n);
    const double y = ldexp(m, e - q * n);
    double t = 2.0;
    for (int it = 0; it < 64; ++it) {
        double p = t;
        for (int i = 2; i < n; ++i) p = p * t; /* t^(n-1) */
        const double tn = ((double)(n - 1) * t + y / p) / (double)n;
        if (!(tn < t)) break;
        t = tn;
    }
    return ldexp(t, q);
}

/* natural log of a positive normal finite x: x = m 2^e, m in [sqrt(1/2), sqrt(2)),
 * log m = 2 atanh(s), s = (m - 1) / (m + 1), |s| <= 0.1716, by its odd series to s^27
 * (truncation < 1e-21 relative), plus e ln 2 in two parts */
RS_FN double rs_log(double x) {
    int e;
    double m = frexp(x, &e);
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e = e - 1;
    }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double t = 1.0 / 27.0;
    for (int k = 25; k >= 1; k -= 2) t = t * s2 + 1.0 / (double)k;
    const double lm = 2.0 * s * t;
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33; /* e * ln2_hi exact */
    return (double)e * ln2_hi + ((double)e * ln2_lo + lm);
}

/* x^m, m >= 1, by m - 1 multiplications in order */
RS_FN double rs_powi(double x, int m) {
    double r = x;
    for (int i = 1; i < m; ++i) r = r * x;
    return r;
}

/* |(x, y)| for the Hartley normalisation (pixel offsets: no overflow to guard) */
RS_FN double rs_hypot(double x, double y) { return sqrt(x * x + y * y); }

/* RANSACUpdateNumIters (calib3d/ptsetreg.cpp); cvRound = round half to even */
RS_FN int rs_update_iters(double p, double ep, int model_points, int max_iters) {
    p = fmin(fmax(p, 0.0), 1.0);
    ep = fmin(fmax(ep, 0.0), 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - rs_powi(1.0 - ep, model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = rs_log(num);
    denom = rs_log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

#endif
