// bdpt_math.h -- the transcendental / root functions of the render path with the exact results
// the oracle's contract requires, cheaper than the generic library sequences.
//
//  * bdpt_sincos_dp: fp64 sin & cos (Cody-Waite reduction by pi/2 with a 33-bit head, fdlibm's
//    degree-13/14 minimax kernels, explicit fma).  Only ever called on x = 2*pi*u with u an MT607
//    float; tests/test_math.py sweeps every float such an x can take (2^28 of them) and checks that
//    (float)result equals (float)sin((double)x) / (float)cos((double)x) of glibc for all of them.
//    Host+device so the same code is what the test runs.
//  * bdpt_sqrt_rn (device): correctly rounded fp32 sqrt = v_sqrt_f32 plus the +-1 ulp residual
//    correction; inputs below 2^-96 (and 0, NaN, negatives) take the library sequence on an
//    exec-masked branch, so the result equals sqrtf() for every input.
#ifndef BDPT_MATH_H
#define BDPT_MATH_H

#ifndef __HIPCC_RTC__
#include <math.h>
#endif

#include "bdpt_sincos_table.h"

#if defined(__HIPCC__)
#define BDPT_HD __host__ __device__ __forceinline__
#else
#define BDPT_HD static inline
#endif

BDPT_HD void bdpt_sincos_dp(double x, double* so, double* co) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double P1 = 1.57079632673412561417e+00;   // pi/2, first 33 bits: k*P1 is exact
    const double P1T = 6.07710050650619224932e-11;  // pi/2 - P1
    const double k = rint(x * 0.63661977236758134308);
    const int q = (int)k;
    const double r = fma(-k, P1T, fma(-k, P1, x));  // x - k*P1 exact (Sterbenz), then the tail
    const double z = r * r;
    const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2), S1);
    const double s = fma(r * z, ps, r);
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * z * pc);
    const double sn = (q & 1) ? c : s, cs = (q & 1) ? s : c;
    *so = (q & 2) ? -sn : sn;
    *co = ((q + 1) & 2) ? -cs : cs;
}

// Table-driven fp64 sin & cos, cheaper than bdpt_sincos_dp (no quadrant logic, short
// polynomials): k = rint(x * N/2pi), r = x - k*2pi/N (two-part constant, |r| <= pi/N),
// sin x = S_k cos r + C_k sin r, cos x = C_k cos r - S_k sin r with S_k = sintab[k] =
// sin(2pi k/N) and C_k = cos(2pi k/N) = sintab[(k + N/4) mod N] (bdpt_sincos_table.h, N = 512,
// correctly rounded, so the two are the same double; the four axis entries exact).  With
// |r| <= pi/512 the Taylor terms r^7/7! and r^6/6! are dropped (sin r = r - r^3/6 + r^5/120,
// cos r = 1 - r^2/2 + r^4/24).  The dropped sine term is below 2^-61 relative, but r^6/6! reaches
// 7.4e-17 = 2^-53.6 -- about 0.67 ulp of cos r ~ 1 -- so the fp64 cos r is NOT accurate to a few
// ulp by this argument alone, and no error bound is claimed here: exactness of the float results
// rests on the exhaustive test (every float x = 2pi u the render path can pass, both tables,
// tests/test_math.py), which must be re-run after any edit to the table, the reduction or the
// polynomials.  For 0 <= x <= 2pi (the render path's x = 2pi u).  BDPT_SC_COARSE = 1: the even
// entries only (N = 256, 2 KB of LDS instead of 4 KB, for kernels whose LDS bounds the
// workgroups per CU); then r^6/6! is kept in cos r.
#ifndef BDPT_SC_COARSE
#define BDPT_SC_COARSE 0
#endif
BDPT_HD void bdpt_sincos_tab(double x, const double* sintab, double* so, double* co) {
#if BDPT_SC_COARSE
    // every other entry (N/2 = 256, 2 KB: LDS-bound kernels), |r| <= pi/256: cos r keeps r^6/6!
    const int NT = BDPT_SC_N / 2;
    const double kd = rint(x * (0.5 * BDPT_SC_INV));
    const int k = ((int)kd) & (NT - 1);
    const double r = fma(-kd, 2.0 * BDPT_SC_C2, fma(-kd, 2.0 * BDPT_SC_C1, x));
    const double z = r * r;
    const double sr = fma(r * z, fma(z, 1.0 / 120.0, -1.0 / 6.0), r);
    const double cr = fma(z, fma(z, fma(z, -1.0 / 720.0, 1.0 / 24.0), -0.5), 1.0);
#else
    const int NT = BDPT_SC_N;
    const double kd = rint(x * BDPT_SC_INV);
    const int k = ((int)kd) & (NT - 1);               // k = N is x = 2pi: entry 0
    const double r = fma(-kd, BDPT_SC_C2, fma(-kd, BDPT_SC_C1, x));
    const double z = r * r;
    const double sr = fma(r * z, fma(z, 1.0 / 120.0, -1.0 / 6.0), r);
    const double cr = fma(z, fma(z, 1.0 / 24.0, -0.5), 1.0);
#endif
    const double S = sintab[k], C = sintab[(k + NT / 4) & (NT - 1)];
    *so = fma(S, cr, C * sr);
    *co = fma(C, cr, -(S * sr));
}

#ifndef BDPT_SQRT_SHIFT
#define BDPT_SQRT_SHIFT 1
#endif
#if defined(__HIPCC__)
// v_sqrt_f32 + the +-1 ulp residual correction: correctly rounded for x >= 2^-96 and x == 0.
__device__ __forceinline__ float bdpt_sqrt_rn_core(float x) {
#if BDPT_SQRT_SHIFT
    // The same decision without VCC selects (+5 % on the path kernel with the det test dropped,
    // bdpt_kernels.hip sphere_isect_inf): the residuals are taken with the opposite sign,
    // r' = fl(s*n - x), so "x <= sdn*s" / "x > sup*s" are sign bits (an exact zero is +0 in
    // round-to-nearest), and s = sdn + [x <= sdn*s is false] + [x > sup*s] (the two conditions
    // exclude each other).  sdn saturates at 0 for s = +0 (then x = 0: both sign bits are 0).
    // Checked against the select form and (float)sqrt((double)x) on all 2^32 inputs on gfx950
    // (scripts/sqrt_shift_check.hip): equal for x = +0 and every x >= 2^-96; a NaN for negative
    // normal x and generated (canonical) NaNs; a NaN or -0 for -0 and negative denormals.
    {
        const unsigned sb = __float_as_uint(__builtin_amdgcn_sqrtf(x));
        const unsigned db = __builtin_elementwise_sub_sat(sb, 1u);
        const float rdn = __builtin_fmaf(__uint_as_float(db), __uint_as_float(sb), -x);
        const float rup = __builtin_fmaf(__uint_as_float(sb + 1u), __uint_as_float(sb), -x);
        return __uint_as_float(db + (__float_as_uint(rdn) >> 31) + (__float_as_uint(rup) >> 31));
    }
#endif
    float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __int_as_float(__float_as_int(s) - 1);
    const float sup = __int_as_float(__float_as_int(s) + 1);
    const float rdn = __builtin_fmaf(-sdn, s, x);
    const float rup = __builtin_fmaf(-sup, s, x);
    // the select form (BDPT_SQRT_SHIFT=0: the reference decision scripts/sqrt_shift_check.hip
    // compares the sign-bit form with)
    s = rdn <= 0.f ? sdn : s;
    s = rup > 0.f ? sup : s;
    return s;
}

__device__ __forceinline__ float bdpt_sqrt_rn(float x) {
    if (__builtin_expect(!(x >= 0x1p-96f), 0)) return sqrtf(x);
    return bdpt_sqrt_rn_core(x);
}
#endif

#endif
