// pm_model.hpp — the point-mass plugin's step (the a16 bring-up dynamics and quadratic cost), the
// one definition both point-mass paths use: pm_rollout_kernel (kernels.hip, the five launches) and
// pm_update_kernel (pm_fused.hip, one launch).  The operation order is explicit and contraction is
// off in every helper, with plain operators inside that scope: HIP's __dmul_rn / __dadd_rn are
// header-inline operators that carry the header's contraction flag, and the backend fused gamma *
// cost + J where the product had one use (the fused kernel) but not where isnan() also read it (the
// five launches): one cost in a thousand differed by an ulp.  So the two paths give the same bits.
//
// A step of the reference's point mass (J += gamma_k cost(x, u); v += u / m dt; p += v dt) splits
// into the part that depends on the state, which is a chain through the horizon, and the part that
// depends on the control alone: the control cost r . u^2 and the velocity increment (u / m) dt.
// The fused launch forms the control part of every (rollout, step) in parallel before the rollouts
// (pm_control_step), so the chain keeps 18 fp64 operations per step.
#pragma once

#include <hip/hip_runtime.h>

#include "engine_types.hpp"

namespace mppi_eng {

// sum_i q_i (p_i - target_i)^2, as fma(q2, d2^2, fma(q1, d1^2, q0 d0^2))
__device__ __forceinline__ double pm_state_cost(const DevPointMass &P, const double *x)
{
#pragma clang fp contract(off)
    const double d0 = x[0] - P.target[0], d1 = x[1] - P.target[1], d2 = x[2] - P.target[2];
    const double e0 = d0 * d0, e1 = d1 * d1, e2 = d2 * d2;
    return __builtin_fma(P.q[2], e2, __builtin_fma(P.q[1], e1, P.q[0] * e0));
}

// sum_i r_i u_i^2, the same association
__device__ __forceinline__ double pm_control_cost(const DevPointMass &P, const double *u)
{
#pragma clang fp contract(off)
    const double e0 = u[0] * u[0], e1 = u[1] * u[1], e2 = u[2] * u[2];
    return __builtin_fma(P.r[2], e2, __builtin_fma(P.r[1], e1, P.r[0] * e0));
}

// the control part of a step: the velocity increments (u_i / m) dt and the control cost
__device__ __forceinline__ void pm_control_step(const DevPointMass &P, const double *u, double dt, double *dv, double &cu)
{
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 3; i++) dv[i] = (u[i] * P.inv_mass) * dt;
    cu = pm_control_cost(P, u);
}

// the state part: the step cost gamma_k (state cost + cu) added to J as a rounded product (no fma),
// then v += dv, p += v dt (mppi.cpp:322-337; the point-mass plugin's step)
__device__ __forceinline__ double pm_state_step(const DevPointMass &P, double *x, const double *dv, double cu, double gamma,
                                                double dt, double &J)
{
#pragma clang fp contract(off)
    const double sc = gamma * (pm_state_cost(P, x) + cu);
    J = J + sc;
#pragma unroll
    for (int i = 0; i < 3; i++) x[3 + i] = x[3 + i] + dv[i];
#pragma unroll
    for (int i = 0; i < 3; i++) x[i] = __builtin_fma(x[3 + i], dt, x[i]);
    return sc;
}

}  // namespace mppi_eng
