/*
 * pt_libm.h — a tiny deterministic libm (sinf / cosf / sincosf / pow(x, 5)) that gives the
 * SAME bits on the x86 host (gcc / g++) and on gfx950 (hipcc device code).
 *
 * Why it exists: the reference's BSDFs call sinf/cosf/powf (interactions.cu:74-75, 201, 253,
 * 260; pathtrace.cu:236).  The reference binary used CUDA libdevice; a host restatement uses
 * glibc; HIP device code would use ocml.  All three differ in the last ulp, and a Monte-Carlo
 * path is chaotic, so a 1-ulp difference re-routes a path.  Both the oracle (in its
 * "portable" trig mode) and the HIP kernels call these functions, so oracle-vs-GPU parity
 * can be checked BIT-EXACTLY; the oracle's "libm" mode (glibc) is what is compared with the
 * reference-derived known answers, within the statistical tolerance of SURVEY §8c.
 *
 * Method (sincos):
 *   |x| < 8 (every argument the path tracer passes: the BSDF and lens angles lie in
 *   [-pi/4, 2 pi)) — FLOAT arithmetic only: k = rint(x 2/pi), a 4-part Cody–Waite reduction
 *   r = x - k pi/2 (1.5703125 + 4.8375129699707031e-4 + 7.5497901264e-8 - 1.7151245e-15, the
 *   first two with trailing zero bits so k*P is exact), and the cephes sinf / cosf minimax
 *   polynomials on [-pi/4, pi/4] (public-domain coefficients), all in EXPLICIT fused
 *   multiply-adds.  Checked exhaustively over every float of (-8, 8) against sin / cos in double
 *   (round 3): max error 1.49 ulp (sin) and 1.55 ulp (cos), CUDA's sinf / cosf class of accuracy.
 *   Round 2 evaluated this range in double (below); FP64 is half rate on gfx950 and the double
 *   version cost 4.6 % of the headline frame (a duplicated call, A/B).
 *   |x| >= 8, inf, NaN — promote to double, Cody–Waite reduce by pi/2 with fdlibm's 3-part
 *   constant, evaluate fdlibm's __kernel_sin / __kernel_cos, round once to float (< 0.5 ulp +
 *   2^-40 relative).
 * fma is exactly specified by IEEE 754, so the host's fma()/fmaf() and gfx950's v_fma_f32 /
 * v_fma_f64 return the same bits; every other operation is a plain IEEE op.  Callers MUST
 * compile with -ffp-contract=off so no further FMA is formed on either side.  The results are
 * therefore identical on both sides.
 *
 * This is test/product shared *libm*, not part of the reference algorithm.
 */
#ifndef PT_LIBM_H
#define PT_LIBM_H

#if defined(__HIPCC__)
#define PT_LIBM_FN __host__ __device__ static inline
#else
#define PT_LIBM_FN static inline
#endif

PT_LIBM_FN double pt_libm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

PT_LIBM_FN double pt_libm_floor(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_floor(x);
#else
    return __builtin_floor(x);
#endif
}

PT_LIBM_FN double pt_kernel_sin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double p = pt_libm_fma(z, S6, S5);
    p = pt_libm_fma(z, p, S4);
    p = pt_libm_fma(z, p, S3);
    p = pt_libm_fma(z, p, S2);
    p = pt_libm_fma(z, p, S1);
    return pt_libm_fma(x * z, p, x);
}

PT_LIBM_FN double pt_kernel_cos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double p = pt_libm_fma(z, C6, C5);
    p = pt_libm_fma(z, p, C4);
    p = pt_libm_fma(z, p, C3);
    p = pt_libm_fma(z, p, C2);
    p = pt_libm_fma(z, p, C1);
    return pt_libm_fma(z * z, p, pt_libm_fma(-0.5, z, 1.0));
}

/* sin and cos of a float: the float-only path for |x| < 8, the double path otherwise. */
PT_LIBM_FN void pt_sincosf_f32(float x, float* s_out, float* c_out) {
    const float INV_PIO2 = 0.636619772367581343f;
    const float P1 = 1.5703125f;                  /* pi/2 = P1 + P2 + P3 + P4 */
    const float P2 = 4.837512969970703125e-4f;
    const float P3 = 7.549790126404332e-08f;
    const float P4 = -1.7151245100058819e-15f;
    const float k = __builtin_rintf(x * INV_PIO2) + 0.0f;   /* + 0: -0 -> +0, so r keeps x's zero sign */
    float r = __builtin_fmaf(-k, P1, x);
    r = __builtin_fmaf(-k, P2, r);
    r = __builtin_fmaf(-k, P3, r);
    r = __builtin_fmaf(-k, P4, r);
    const float z = r * r;
    const float s = __builtin_fmaf(
        __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
    const float c = __builtin_fmaf(
        __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f) * z,
        z, __builtin_fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    float so = (q & 1) ? c : s, co = (q & 1) ? s : c;
    if (q == 1 || q == 2) co = -co;
    if (q == 2 || q == 3) so = -so;
    *s_out = so;
    *c_out = co;
}
PT_LIBM_FN void pt_sincosf(float xf, float* s_out, float* c_out) {
    if (__builtin_fabsf(xf) < 8.0f) {
        pt_sincosf_f32(xf, s_out, c_out);
        return;
    }
    double x = (double)xf;
    double ax = x < 0.0 ? -x : x;
    if (!(ax < 1.0e9)) {            /* inf / NaN / absurdly large: NaN like libm for inf/NaN */
        float nan = xf - xf;
        if (ax == ax && ax >= 1.0e9) nan = 0.0f / 0.0f;
        *s_out = nan;
        *c_out = nan;
        return;
    }
    const double INV_PIO2 = 6.36619772367581382433e-01;
    const double PIO2_1 = 1.57079632673412561417e+00;   /* first 33 bits of pi/2 */
    const double PIO2_2 = 6.07710050630396597660e-11;   /* next 33 bits */
    const double PIO2_3 = 2.02226624871116645580e-21;   /* next 33 bits */
    const double PIO2_3T = 8.47842766036889956997e-32;  /* tail */
    double k = pt_libm_floor(pt_libm_fma(x, INV_PIO2, 0.5));
    double r = pt_libm_fma(-k, PIO2_1, x);    /* k < 2^30: each step exact up to the last rounding */
    r = pt_libm_fma(-k, PIO2_2, r);
    r = pt_libm_fma(-k, PIO2_3, r);
    r = pt_libm_fma(-k, PIO2_3T, r);
    long long ki = (long long)k;
    int q = (int)(ki & 3);
    double s = pt_kernel_sin(r);
    double c = pt_kernel_cos(r);
    double so, co;
    switch (q) {
        case 0: so = s; co = c; break;
        case 1: so = c; co = -s; break;
        case 2: so = -s; co = -c; break;
        default: so = -c; co = s; break;
    }
    *s_out = (float)so;
    *c_out = (float)co;
}

PT_LIBM_FN float pt_sinf(float x) { float s, c; pt_sincosf(x, &s, &c); return s; }
PT_LIBM_FN float pt_cosf(float x) { float s, c; pt_sincosf(x, &s, &c); return c; }

/* powf(x, 5.0f) as used by FresnelSchlick (interactions.cu:197-201): x^5 in double, one rounding. */
PT_LIBM_FN float pt_pow5f(float xf) {
    double x = (double)xf;
    double x2 = x * x;
    double x4 = x2 * x2;
    return (float)(x4 * x);
}

#endif /* PT_LIBM_H */
