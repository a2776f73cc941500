// fsincos.hpp — branch-free sin / cos of a joint angle (fdlibm kernels), shared by the rollout
// kernel (fr_coop.hip) and the objective kernel (fr_cost.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace mppi_eng {

// fdlibm's __kernel_sin / __kernel_cos coefficients, held in SGPRs for the horizon loop: built once
// and made opaque, so the loop's FMAs read them as scalar operands instead of rematerialising each
// as two v_mov_b32 per step (machine LICM stays off for this file, see the Makefile)
struct SinCosK {
    double s[6], c[6];
};
__device__ __forceinline__ SinCosK sincos_constants()
{
    SinCosK k{{-1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,
               2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10},
              {4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,
               -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11}};
#pragma unroll
    for (int i = 0; i < 6; i++)
        if (i != 4) asm volatile("" : "+s"(k.s[i]), "+s"(k.c[i]));
    // the innermost Horner FMAs fma(z, s5, s4) would read two scalar operands (one allowed): s4 and
    // c4 live in VGPRs, instead of a v_mov_b64 of each per use (two per rollout step, r05)
    asm volatile("" : "+v"(k.s[4]), "+v"(k.c[4]));
    return k;
}

// sin and cos of a joint angle, branch-free (the library sincos branches to a Payne-Hanek
// reduction for |x| >= 2^30, which ended the step's last scheduling region).  Valid for
// |x| < 2^26: k = rint(2x / pi), r = x - k pi/2 with pi/2 in two parts (the first FMA is exact
// for these k), fdlibm's __kernel_sin / __kernel_cos polynomials on [-pi/4, pi/4] (< 1 ulp), and
// the quadrant by selects and a sign flip.  Joint angles are O(10); inf / NaN give NaN as sin does.
__device__ __forceinline__ void fsincos(double x, double *sp, double *cp, const SinCosK &K)
{
    const double k = __builtin_rint(x * 0.63661977236758134308);
    double r = __builtin_fma(-k, 1.5707963267948966, x);
    r = __builtin_fma(-k, 6.123233995736766e-17, r);
    const double z = r * r;
    const double ps = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                      __builtin_fma(z, K.s[5], K.s[4]), K.s[3]), K.s[2]), K.s[1]), K.s[0]);
    const double s = __builtin_fma(r * z, ps, r);
    const double pc = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                      __builtin_fma(z, K.c[5], K.c[4]), K.c[3]), K.c[2]), K.c[1]), K.c[0]);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + (z * z) * pc);
    const int n = (int)k;
    const bool swap = (n & 1) != 0;
    const double sv = swap ? c : s, cv = swap ? s : c;
    *sp = __hiloint2double(__double2hiint(sv) ^ (int)((unsigned)(n & 2) << 30), __double2loint(sv));
    *cp = __hiloint2double(__double2hiint(cv) ^ (int)((unsigned)((n + 1) & 2) << 30), __double2loint(cv));
}

}  // namespace mppi_eng
