// ctr_math.hpp -- fp64 elementary functions for the CTR kernels (host + device).
//
// sincos_cw: Cody-Waite reduction by pi/2 (three FMA terms) + fdlibm-style minimax kernels on
// [-pi/4, pi/4]; sine and cosine share one reduction.  Arguments beyond |x| < 2^20 (never
// reached by joint angles, which are bounded by the action limits and episode length) fall
// back to the math library.  Max error <= 2 ulp is checked on the host by tests/test_math.py.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define CTR_HD __host__ __device__ __forceinline__
#else
#define CTR_HD static inline
#endif

namespace ctr_math {

struct SinCos {
    double s, c;
};

// Out-of-line slow path (keeps the math library's large-argument reduction out of every
// inlined call site).  Returns by value so callers keep their operands in registers.
#if defined(__HIPCC__)
__host__ __device__ __attribute__((noinline))
#else
static
#endif
SinCos sincos_slow(double x)
{
    SinCos r;
    r.s = sin(x);
    r.c = cos(x);
    return r;
}

// Fast path only (valid for |x| < 2^20): Cody-Waite + minimax kernels, branch-free.
CTR_HD void sincos_fast(double x, double &sv, double &cv)
{
    const double n = rint(x * 0.6366197723675814);             // round(x * 2/pi)
    double r = fma(-n, 1.5707963267948966, x);                 // pi/2 = P1 + P2 + P3
    r = fma(-n, 6.123233995736766e-17, r);
    r = fma(-n, -1.4973849048591698e-33, r);
    const double z = r * r;
    // Estrin evaluation of the same minimax kernels: dependency depth 3 instead of 5-6 (one
    // wave per SIMD exposes fp64 FMA latency)
    const double z2 = z * z;
    const double sa = fma(z, -1.98412698298579493134e-04, 8.33333333332248946124e-03);
    const double sb = fma(z, -2.50507602534068634195e-08, 2.75573137070700676789e-06);
    const double ps = fma(z2, fma(z2, 1.58969099521155010221e-10, sb), sa);
    const double s = r + (z * r) * (-1.66666666666666324348e-01 + z * ps);
    const double ca = fma(z, -1.38888888888741095749e-03, 4.16666666666666019037e-02);
    const double cb = fma(z, -2.75573143513906633035e-07, 2.48015872894767294178e-05);
    const double c3 = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    const double pc = z * fma(z2, fma(z2, c3, cb), ca);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * pc);
    const int q = ((int)n) & 3;
    const double ss = (q & 1) ? c : s;
    const double cc = (q & 1) ? s : c;
    sv = (q & 2) ? -ss : ss;
    cv = ((q + 1) & 2) ? -cc : cc;
}

CTR_HD bool sincos_needs_slow(double x) { return !(fabs(x) < 1048576.0); }

// Table-based sincos: x = n (pi/256) + r, |r| <= pi/512, with (sin, cos)(k pi/256), k = n mod 512,
// from an 8 KB table (kept in LDS by the kernels) and short Taylor kernels on r:
//   sin x = S_k cos r + C_k sin r,   cos x = C_k cos r - S_k sin r.
// Degree 5 / 4 kernels (truncation < 7e-20 relative for sin, < 7.4e-17 absolute for cos) and a
// two-term Cody-Waite reduction (the third pi/256 term is below 1e-28 for |x| < 2^20): 14 fp64
// operations per angle, no quadrant selects.  One wave per SIMD makes the FK loop issue-bound,
// so every operation counts (the pi/64 table with degree-7 / 6 kernels took 16).  Max error
// <= 2 ulp (tests/test_math.py).  Valid for |x| < 2^20 like sincos_fast.
#include "ctr_trig_tab512.inc"

// Split in two so callers can issue the reduction and the table loads a stage ahead of the
// polynomial work that consumes them (one wave per SIMD cannot hide the LDS latency otherwise).
struct TabPre {
    double r0, r1;               // reduced arguments, |r| <= pi/512
    double ts0, tc0, ts1, tc1;   // (sin, cos)(k pi/256) of each angle
};

CTR_HD TabPre sincos_tab2_pre(double x0, double x1, const double (*tab)[2])
{
    TabPre p;
    const double n0 = rint(x0 * 81.48733086305042), n1 = rint(x1 * 81.48733086305042);   // round(x 256/pi)
    const int k0 = ((int)n0) & 511, k1 = ((int)n1) & 511;
    p.ts0 = tab[k0][0];
    p.tc0 = tab[k0][1];
    p.ts1 = tab[k1][0];
    p.tc1 = tab[k1][1];
    p.r0 = fma(-n0, 4.783776559169348e-19, fma(-n0, 0.01227184630308513, x0));
    p.r1 = fma(-n1, 4.783776559169348e-19, fma(-n1, 0.01227184630308513, x1));
    return p;
}

CTR_HD void sincos_tab2_post(const TabPre &p, double &s0, double &c0, double &s1, double &c1)
{
    const double r0 = p.r0, r1 = p.r1;
    const double z0 = r0 * r0, z1 = r1 * r1;
    // sin r = r + r z (-1/6 + z / 120),  cos r = 1 + z (-1/2 + z / 24)
    const double sp0 = fma(z0, 8.3333333333333332e-03, -1.6666666666666666e-01);
    const double sp1 = fma(z1, 8.3333333333333332e-03, -1.6666666666666666e-01);
    const double cp0 = fma(z0, 4.1666666666666664e-02, -0.5);
    const double cp1 = fma(z1, 4.1666666666666664e-02, -0.5);
    const double sr0 = fma(r0 * z0, sp0, r0), sr1 = fma(r1 * z1, sp1, r1);
    const double cr0 = fma(z0, cp0, 1.0), cr1 = fma(z1, cp1, 1.0);
    s0 = fma(p.ts0, cr0, p.tc0 * sr0);
    c0 = fma(p.tc0, cr0, -(p.ts0 * sr0));
    s1 = fma(p.ts1, cr1, p.tc1 * sr1);
    c1 = fma(p.tc1, cr1, -(p.ts1 * sr1));
}

CTR_HD void sincos_tab2(double x0, double x1, const double (*tab)[2], double &s0, double &c0, double &s1,
                        double &c1)
{
    sincos_tab2_post(sincos_tab2_pre(x0, x1, tab), s0, c0, s1, c1);
}

CTR_HD void sincos_tab(double x, const double (*tab)[2], double &sv, double &cv)
{
    double s1, c1;
    sincos_tab2(x, 0.0, tab, sv, cv, s1, c1);
}


CTR_HD void sincos_cw(double x, double *sp, double *cp)
{
    if (sincos_needs_slow(x)) {                   // rare: huge or non-finite arguments
        const SinCos r = sincos_slow(x);
        *sp = r.s;
        *cp = r.c;
        return;
    }
    sincos_fast(x, *sp, *cp);
}

// 1/x to within 1 ulp: hardware reciprocal estimate + two Newton-Raphson steps.
CTR_HD double rcp(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
#else
    return 1.0 / x;
#endif
}

// max(|a|, |b|) as one v_max_f64 with abs modifiers (fmax() would first canonicalize each
// loop-carried operand with an extra v_max: the error scales of the step controller).
CTR_HD double absmax(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmax(fabs(a), fabs(b));
#endif
}

// 1/x to about 1 ulp with a single Newton-Raphson step (step-size control only).
CTR_HD double rcp1(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double r = __builtin_amdgcn_rcp(x);
    return fma(r, fma(-x, r, 1.0), r);
#else
    return 1.0 / x;
#endif
}

// 1/x as the bare v_rcp_f64 estimate (relative error <= 2^-24, tools/ubench/rcp_acc: max 2.6e8 ulp).
// Used only for the 18 error scales 1/(atol + |y| rtol) of the RK45 step controller: the error
// norm, and from it the accept/reject decision and the next step size, then carry a relative
// error below 6e-8, which moves h by < 1.2e-8 relative (the tip by ~1e-12 m) and flips an
// accept/reject decision only when the norm is within 6e-8 of 1.
CTR_HD double rcp_est(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(x);
#else
    return 1.0 / x;
#endif
}

// x^(-1/10) for finite x > 0, ~1 ulp: x = x' 2^(10k) with x' in [1, 2^10); a float32
// exp2/log2 seed for x'^(-1/10), two float64 Newton steps on y^10 x' = 1, then 2^(-k).
// (Replaces pow(), ~5x cheaper; used by the RK45 step-size controller only.)
CTR_HD double inv_root10(double x)
{
    int e;
    const double m = frexp(x, &e);                       // x = m 2^e, m in [0.5, 1)
    // write e - 1 = 10 k + r with r in [0, 10)
    const int em1 = e - 1;                               // >= -1075 (subnormals), so em1 + 1100 >= 0:
    const int k = (int)((unsigned)(em1 + 1100) / 10u) - 110;   // floor((e - 1) / 10), no branch
    const int r = em1 - 10 * k;
    const double xs = ldexp(m, r + 1);                   // x' = x 2^(-10k) in [1, 2^10)
#if defined(__HIP_DEVICE_COMPILE__)
    const float sf = __builtin_amdgcn_exp2f(-0.1f * __builtin_amdgcn_logf((float)xs));
#else
    const float sf = exp2f(-0.1f * log2f((float)xs));
#endif
    double y = (double)sf;
    #pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double y2 = y * y, y4 = y2 * y2, y8 = y4 * y4;
        const double t = xs * (y8 * y2);                 // x' y^10 ~ 1
        y = y + y * ((1.0 - t) * 0.1);                   // y (1 + (1 - t)/10)
    }
    return ldexp(y, -k);
}

// nextafter(t, +inf) - t, exactly, without nextafter's integer bit manipulation (a power of two:
// 2^(e-53) for |t| = m 2^e, m in [0.5, 1), half that for a negative power of two, 2^-1074 at and
// below the subnormal spacing); NaN for NaN and +inf, +inf for -inf and the largest double, as
// nextafter(t, inf) - t.
CTR_HD double gap_up(double t)
{
    int e;
    const double m = frexp(t, &e);
    const int sh = (m == -0.5) ? 54 : 53;
    const int p = e - sh;
    double g = ldexp(1.0, p < -1074 ? -1074 : p);
    g = (t == 0.0) ? 4.9406564584124654e-324 : g;
    return (t == -INFINITY || t == 1.7976931348623157e308) ? INFINITY : g + 0.0 * t;
}

// sqrt(x) for finite x > 0, ~1 ulp: reciprocal square root estimate + Newton (no division).
CTR_HD double sqrt_rsq(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rsq(x);
#else
    double r = 1.0 / sqrt(x);
#endif
    r = r * fma(-0.5 * x, r * r, 1.5);
    double s = x * r;
    return fma(0.5 * r, fma(-s, s, x), s);
}

// x^y for x > 0 through exp2/log2 (step-size factors only; a few ulp).
CTR_HD double powpos(double x, double y)
{
    return exp2(y * log2(x));
}

}  // namespace ctr_math
