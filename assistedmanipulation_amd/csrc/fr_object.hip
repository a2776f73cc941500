// fr_object.hip — FrankaRidgeback::PinocchioDynamics as one device-resident object (a single
// trajectory), and AssistedManipulation / TrackPoint get_cost evaluated against it.
//
// The reference's plugin objects are used outside mppi::Trajectory too: the Actor's
// DynamicsForecast rolls its own PinocchioDynamics forward with zero control every controller
// period (frankaridgeback/dynamics.cpp:104-138, actor.cpp:176-177), and a plugin is an object with
// set_state / step / get_state / get_end_effector_state (mppi.hpp:47-84, dynamics.hpp:416-537).
// This file keeps that object's state in HBM and runs its methods as one-thread kernels (one
// launch per call; forecast() one launch for the whole horison): latency-bound by nature, nothing
// to spread over a wave, and not on the rollout path (the rollouts run in fr_coop.hip).
//
// Semantics follow pinocchio_dynamics.cpp:142-260 literally, quirks included:
//   set_state   q, v, tank energy from the state; calculate() with m_joint_torque += NLE(q, v) on
//               the torque left by the previous call (so the acceleration after a set_state is
//               M^-1 tau_stale);
//   step        base velocity overwritten by R(yaw) u[0:2], u[2]; tau = 0 but the arm's u[3:10];
//               calculate(): tau += NLE, a = aba(q, v, tau) = M^-1 tau_u; v += a dt, q += v dt;
//               power = tau . v, EnergyTank::step (energy.hpp:19-22);
//   calculate   FK with (q, v, a), the EE frame (panda_grasp_joint) placement, its WORLD Jacobian
//               with the top-left 3x3 overwritten by R_z(yaw), its WORLD spatial velocity and
//               acceleration (pinocchio_dynamics.cpp:153-224), the arm-mount frame position.
// Arithmetic is the world-frame form of the rollout kernels: RNEA for NLE, and M^-1 by the
// composite-rigid-body algorithm and a Cholesky solve (rounding differs from Pinocchio's ABA).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "fr_cost_terms.hpp"

using namespace mppi_eng;

namespace {

__device__ __forceinline__ void cross3(const double *a, const double *b, double *o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ double dot6(const double *a, const double *b)
{
    return ((a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3])) + (a[4] * b[4] + a[5] * b[5]);
}
// motion cross product [v; w] x [x_v; x_w] = [w x x_v + v x x_w; w x x_w]
__device__ __forceinline__ void motion_cross(const double *V, const double *X, double *o)
{
    double a[3], b[3];
    cross3(V + 3, X, a);
    cross3(V, X + 3, b);
    cross3(V + 3, X + 3, o + 3);
    for (int k = 0; k < 3; k++) o[k] = a[k] + b[k];
}

// Kinematics of one configuration, world frame at the origin: body poses and motion subspaces,
// each body's mass, world com and rotational inertia about it.
struct Bodies {
    double R[FR_NB][9], p[FR_NB][3], S[FR_NB][6], c[FR_NB][3], Iw[FR_NB][6];   // Iw: xx xy xz yy yz zz
};

__device__ void fk_bodies(const DevModel &M, const double *q, Bodies &B)
{
    for (int i = 0; i < FR_NB; i++) {
        const DevBody &b = M.b[i];
        double Rl[9], pl[3];
        if (FR_KIND[i] == KIND_RZ) {
            const double s = sin(q[i]), c = cos(q[i]);
            for (int r = 0; r < 3; r++) {
                Rl[3 * r + 0] = b.R[3 * r + 0] * c + b.R[3 * r + 1] * s;
                Rl[3 * r + 1] = b.R[3 * r + 0] * (-s) + b.R[3 * r + 1] * c;
                Rl[3 * r + 2] = b.R[3 * r + 2];
                pl[r] = b.p[r];
            }
        } else {
            const int col = FR_KIND[i] == KIND_PX ? 0 : 1;
            const double qq = FR_KIND[i] == KIND_PNY ? -q[i] : q[i];
            for (int r = 0; r < 3; r++) {
                for (int k = 0; k < 3; k++) Rl[3 * r + k] = b.R[3 * r + k];
                pl[r] = b.p[r] + b.R[3 * r + col] * qq;
            }
        }
        const int par = FR_PARENT[i];
        double *R = B.R[i], *p = B.p[i];
        if (par < 0) {
            for (int k = 0; k < 9; k++) R[k] = Rl[k];
            for (int k = 0; k < 3; k++) p[k] = pl[k];
        } else {
            const double *Rp = B.R[par], *pp = B.p[par];
            for (int r = 0; r < 3; r++) {
                for (int cc = 0; cc < 3; cc++) R[3 * r + cc] = (Rp[3 * r] * Rl[cc] + Rp[3 * r + 1] * Rl[3 + cc]) + Rp[3 * r + 2] * Rl[6 + cc];
                p[r] = pp[r] + ((Rp[3 * r] * pl[0] + Rp[3 * r + 1] * pl[1]) + Rp[3 * r + 2] * pl[2]);
            }
        }
        double *S = B.S[i];
        if (FR_KIND[i] == KIND_RZ) {
            const double w[3] = {R[2], R[5], R[8]};
            cross3(p, w, S);
            S[3] = w[0]; S[4] = w[1]; S[5] = w[2];
        } else {
            const int col = FR_KIND[i] == KIND_PX ? 0 : 1;
            const double sg = FR_KIND[i] == KIND_PNY ? -1.0 : 1.0;
            S[0] = sg * R[col]; S[1] = sg * R[3 + col]; S[2] = sg * R[6 + col];
            S[3] = 0.0; S[4] = 0.0; S[5] = 0.0;
        }
        for (int r = 0; r < 3; r++) B.c[i][r] = ((R[3 * r] * b.c[0] + R[3 * r + 1] * b.c[1]) + R[3 * r + 2] * b.c[2]) + p[r];
        // R Ic R^T, Ic from (xx, xy, yy, xz, yz, zz)
        const double I[9] = {b.Ic[0], b.Ic[1], b.Ic[3], b.Ic[1], b.Ic[2], b.Ic[4], b.Ic[3], b.Ic[4], b.Ic[5]};
        double RI[9];
        for (int r = 0; r < 3; r++)
            for (int cc = 0; cc < 3; cc++) RI[3 * r + cc] = (R[3 * r] * I[cc] + R[3 * r + 1] * I[3 + cc]) + R[3 * r + 2] * I[6 + cc];
        int k = 0;
        for (int r = 0; r < 3; r++)
            for (int cc = r; cc < 3; cc++, k++) B.Iw[i][k] = (RI[3 * r] * R[3 * cc] + RI[3 * r + 1] * R[3 * cc + 1]) + RI[3 * r + 2] * R[3 * cc + 2];
    }
}

// body i's spatial inertia (world, at the origin) times a motion [v; w]: [m (v + w x c); Iw w + c x (m (v + w x c))]
__device__ void inertia_mul(const DevModel &M, const Bodies &B, int i, const double *x, double *h)
{
    const double m = M.b[i].mass;
    const double *c = B.c[i], *I = B.Iw[i];
    double wc[3], ch[3];
    cross3(x + 3, c, wc);
    for (int k = 0; k < 3; k++) h[k] = m * (x[k] + wc[k]);
    cross3(c, h, ch);
    h[3] = ((I[0] * x[3] + I[1] * x[4]) + I[2] * x[5]) + ch[0];
    h[4] = ((I[1] * x[3] + I[3] * x[4]) + I[4] * x[5]) + ch[1];
    h[5] = ((I[2] * x[3] + I[4] * x[4]) + I[5] * x[5]) + ch[2];
}

// RNEA (world frame): tau = M(q) qdd + C(q, v) v + g(q); qdd = 0 gives nonLinearEffects.
// Also returns each body's spatial velocity V (the prefix sums the EE frame velocity reads).
__device__ void rnea(const DevModel &M, const Bodies &B, const double *v, const double *qdd, const double *grav, double *tau,
                     double (*V)[6])
{
    double A[FR_NB][6], F[FR_NB][6];
    for (int i = 0; i < FR_NB; i++) {
        const int par = FR_PARENT[i];
        double vj[6], cr[6];
        for (int k = 0; k < 6; k++) vj[k] = B.S[i][k] * v[i];
        double Ap[6] = {-grav[0], -grav[1], -grav[2], 0.0, 0.0, 0.0}, Vp[6] = {0, 0, 0, 0, 0, 0};
        if (par >= 0)
            for (int k = 0; k < 6; k++) { Ap[k] = A[par][k]; Vp[k] = V[par][k]; }
        motion_cross(Vp, vj, cr);
        for (int k = 0; k < 6; k++) {
            V[i][k] = Vp[k] + vj[k];
            A[i][k] = (Ap[k] + B.S[i][k] * qdd[i]) + cr[k];
        }
        double hA[6], hV[6];
        inertia_mul(M, B, i, A[i], hA);
        inertia_mul(M, B, i, V[i], hV);
        double g0[3], g1[3], g2[3];   // V x* h = [w x h_lin; w x h_ang + v x h_lin]
        cross3(V[i] + 3, hV, g0);
        cross3(V[i] + 3, hV + 3, g1);
        cross3(V[i], hV, g2);
        for (int k = 0; k < 3; k++) {
            F[i][k] = hA[k] + g0[k];
            F[i][3 + k] = hA[3 + k] + (g1[k] + g2[k]);
        }
    }
    for (int i = FR_NB - 1; i >= 0; i--) {
        tau[i] = dot6(B.S[i], F[i]);
        const int par = FR_PARENT[i];
        if (par >= 0)
            for (int k = 0; k < 6; k++) F[par][k] += F[i][k];
    }
}

// x = M(q)^-1 b: the mass matrix by the composite-rigid-body algorithm (world frame: a subtree's
// composite inertia is the sum of its bodies' (m, h = m c, I about the origin)), Cholesky solve.
__device__ void solve_mass(const DevModel &M, const Bodies &B, const double *b, double *x)
{
    double m[FR_NB], h[FR_NB][3], I[FR_NB][6];   // composite, I packed xx xy xz yy yz zz
    for (int i = 0; i < FR_NB; i++) {
        const double mi = M.b[i].mass, *c = B.c[i], *Iw = B.Iw[i];
        const double cc2 = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
        m[i] = mi;
        for (int k = 0; k < 3; k++) h[i][k] = mi * c[k];
        I[i][0] = Iw[0] + mi * (cc2 - c[0] * c[0]);
        I[i][1] = Iw[1] - mi * c[0] * c[1];
        I[i][2] = Iw[2] - mi * c[0] * c[2];
        I[i][3] = Iw[3] + mi * (cc2 - c[1] * c[1]);
        I[i][4] = Iw[4] - mi * c[1] * c[2];
        I[i][5] = Iw[5] + mi * (cc2 - c[2] * c[2]);
    }
    for (int i = FR_NB - 1; i > 0; i--) {   // children into parents (bodies 10 and 11 both into 9)
        const int par = FR_PARENT[i];
        m[par] += m[i];
        for (int k = 0; k < 3; k++) h[par][k] += h[i][k];
        for (int k = 0; k < 6; k++) I[par][k] += I[i][k];
    }
    double A[FR_NB][FR_NB];
    for (int j = 0; j < FR_NB; j++) {
        const double *S = B.S[j];
        double F[6];   // Ic_j S_j = [m v - h x w; h x v + I w]
        double hw[3], hv[3];
        cross3(h[j], S + 3, hw);
        cross3(h[j], S, hv);
        for (int k = 0; k < 3; k++) F[k] = m[j] * S[k] - hw[k];
        const double *Ij = I[j];
        F[3] = hv[0] + ((Ij[0] * S[3] + Ij[1] * S[4]) + Ij[2] * S[5]);
        F[4] = hv[1] + ((Ij[1] * S[3] + Ij[3] * S[4]) + Ij[4] * S[5]);
        F[5] = hv[2] + ((Ij[2] * S[3] + Ij[4] * S[4]) + Ij[5] * S[5]);
        for (int i = 0; i < FR_NB; i++) A[i][j] = 0.0;
        for (int i = j; i >= 0; i = FR_PARENT[i]) {   // j and its ancestors
            A[i][j] = dot6(B.S[i], F);
            A[j][i] = A[i][j];
        }
    }
    // Cholesky A = L L^T (in place, lower), then two triangular solves
    for (int j = 0; j < FR_NB; j++) {
        double d = A[j][j];
        for (int k = 0; k < j; k++) d -= A[j][k] * A[j][k];
        const double ljj = sqrt(d);
        A[j][j] = ljj;
        for (int i = j + 1; i < FR_NB; i++) {
            double s = A[i][j];
            for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k];
            A[i][j] = s / ljj;
        }
    }
    double y[FR_NB];
    for (int i = 0; i < FR_NB; i++) {
        double s = b[i];
        for (int k = 0; k < i; k++) s -= A[i][k] * y[k];
        y[i] = s / A[i][i];
    }
    for (int i = FR_NB - 1; i >= 0; i--) {
        double s = y[i];
        for (int k = i + 1; k < FR_NB; k++) s -= A[k][i] * x[k];
        x[i] = s / A[i][i];
    }
}

// PinocchioDynamics::calculate() (pinocchio_dynamics.cpp:153-224) on the object
__device__ void calculate(const DevModel &M, DevPinocchio &P)
{
    Bodies B;
    fk_bodies(M, P.q, B);
    const double zero[FR_NB] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double nle[FR_NB], V[FR_NB][6];
    rnea(M, B, P.v, zero, M.gravity, nle, V);
    double rhs[FR_NB];
    for (int i = 0; i < FR_NB; i++) {
        P.tau[i] += nle[i];          // m_joint_torque += nonLinearEffects (:156-161)
        rhs[i] = P.tau[i] - nle[i];  // aba(q, v, tau) = M^-1 (tau - nle)
    }
    solve_mass(M, B, rhs, P.a);
    // forwardKinematics(q, v, a): spatial accelerations without gravity, A_i = A_par + S_i a_i + V_par x S_i v_i
    double A[FR_NB][6];
    for (int i = 0; i < FR_NB; i++) {
        const int par = FR_PARENT[i];
        double vj[6], cr[6], Vp[6] = {0, 0, 0, 0, 0, 0}, Ap[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 6; k++) vj[k] = B.S[i][k] * P.v[i];
        if (par >= 0)
            for (int k = 0; k < 6; k++) { Vp[k] = V[par][k]; Ap[k] = A[par][k]; }
        motion_cross(Vp, vj, cr);
        for (int k = 0; k < 6; k++) A[i][k] = (Ap[k] + B.S[i][k] * P.a[i]) + cr[k];
    }
    // the end-effector frame on body 9, the arm-mount frame on body 2 (updateFramePlacements)
    double *ee = P.ee;
    const double *R9 = B.R[FR_EE_PARENT], *p9 = B.p[FR_EE_PARENT];
    double Re[9];
    for (int r = 0; r < 3; r++) {
        ee[MPPI_EE_POSITION + r] = p9[r] + ((R9[3 * r] * M.ee_p[0] + R9[3 * r + 1] * M.ee_p[1]) + R9[3 * r + 2] * M.ee_p[2]);
        for (int cc = 0; cc < 3; cc++) Re[3 * r + cc] = (R9[3 * r] * M.ee_R[cc] + R9[3 * r + 1] * M.ee_R[3 + cc]) + R9[3 * r + 2] * M.ee_R[6 + cc];
    }
    for (int k = 0; k < 9; k++) ee[MPPI_EE_ROTATION + k] = Re[k];
    {   // Quaterniond from the rotation matrix (Eigen's quaternionbase_assign_impl), (x, y, z, w)
        double qv[4];
        const double t = (Re[0] + Re[4]) + Re[8];
        if (t > 0.0) {
            double s = sqrt(t + 1.0);
            qv[3] = 0.5 * s;
            s = 0.5 / s;
            qv[0] = (Re[7] - Re[5]) * s;
            qv[1] = (Re[2] - Re[6]) * s;
            qv[2] = (Re[3] - Re[1]) * s;
        } else {
            int i = 0;
            if (Re[4] > Re[0]) i = 1;
            if (Re[8] > Re[4 * i]) i = 2;
            const int j = (i + 1) % 3, k = (j + 1) % 3;
            double s = sqrt(((Re[4 * i] - Re[4 * j]) - Re[4 * k]) + 1.0);
            qv[i] = 0.5 * s;
            s = 0.5 / s;
            qv[3] = (Re[3 * k + j] - Re[3 * j + k]) * s;
            qv[j] = (Re[3 * j + i] + Re[3 * i + j]) * s;
            qv[k] = (Re[3 * k + i] + Re[3 * i + k]) * s;
        }
        for (int k = 0; k < 4; k++) ee[MPPI_EE_QUATERNION + k] = qv[k];
    }
    for (int k = 0; k < 3; k++) {
        ee[MPPI_EE_LINEAR_VELOCITY + k] = V[FR_EE_PARENT][k];
        ee[MPPI_EE_ANGULAR_VELOCITY + k] = V[FR_EE_PARENT][3 + k];
        ee[MPPI_EE_LINEAR_ACCELERATION + k] = A[FR_EE_PARENT][k];
        ee[MPPI_EE_ANGULAR_ACCELERATION + k] = A[FR_EE_PARENT][3 + k];
    }
    double *J = ee + MPPI_EE_JACOBIAN;   // 6 x 12 row-major: columns of the EE's supporting joints
    for (int c = 0; c < FR_NB; c++) {
        const bool support = c <= FR_EE_PARENT;
        for (int r = 0; r < 6; r++) J[r * FR_NB + c] = support ? B.S[c][r] : 0.0;
    }
    const double cy = cos(P.q[2]), sy = sin(P.q[2]);   // topLeftCorner<3, 3> = R_z(yaw) (:196-200)
    J[0] = cy; J[1] = -sy; J[2] = 0.0;
    J[FR_NB] = sy; J[FR_NB + 1] = cy; J[FR_NB + 2] = 0.0;
    J[2 * FR_NB] = 0.0; J[2 * FR_NB + 1] = 0.0; J[2 * FR_NB + 2] = 1.0;
    const double *R2 = B.R[FR_AM_PARENT], *p2 = B.p[FR_AM_PARENT];
    for (int r = 0; r < 3; r++) P.am[r] = p2[r] + ((R2[3 * r] * M.am_p[0] + R2[3 * r + 1] * M.am_p[1]) + R2[3 * r + 2] * M.am_p[2]);
}

__device__ void set_state(const DevModel &M, DevPinocchio &P, const double *x, double time)
{
    P.time = time;
    for (int i = 0; i < FR_X; i++) P.state[i] = x[i];
    for (int i = 0; i < FR_NB; i++) {
        P.q[i] = x[i];
        P.v[i] = x[FR_NB + i];
    }
    P.energy = x[FR_X - 1];   // EnergyTank::set_energy(state.available_energy)
    calculate(M, P);
}

__device__ void step(const DevModel &M, DevPinocchio &P, const double *u, double dt)
{
    const double yaw = P.q[2], c = cos(yaw), s = sin(yaw);
    P.v[0] = c * u[0] + (-s) * u[1];   // Rotation2Dd(yaw) * base_velocity (:234)
    P.v[1] = s * u[0] + c * u[1];
    P.v[2] = u[2];
    for (int i = 0; i < FR_NB; i++) P.tau[i] = (i >= 3 && i < 10) ? u[i] : 0.0;   // segment<ARM>(BASE)
    calculate(M, P);
    for (int i = 0; i < FR_NB; i++) P.v[i] = P.v[i] + P.a[i] * dt;
    for (int i = 0; i < FR_NB; i++) P.q[i] = P.q[i] + P.v[i] * dt;
    double power = 0.0;
    for (int i = 0; i < FR_NB; i++) power += P.tau[i] * P.v[i];
    P.power = power;
    const double e = P.energy + power * dt;
    P.energy = e > 0.0 ? e : 0.0;   // EnergyTank::step: max(0, E + P dt)
    for (int i = 0; i < FR_NB; i++) {
        P.state[i] = P.q[i];
        P.state[FR_NB + i] = P.v[i];
    }
    P.state[FR_X - 1] = P.energy;
    P.time += dt;
}

}  // namespace

// One call of the object's API per launch (ObjOp), one thread.  The forecast row of step k:
// joint position, EndEffectorState, joint power (0), external power (0), tank energy, and the
// wrench forecast(t_k) the caller sampled (DynamicsForecast::forecast, dynamics.cpp:104-138).
__global__ __launch_bounds__(64) void fr_object_kernel(ObjArgs a)
{
    if (threadIdx.x != 0) return;
    DevPinocchio &P = *a.obj;
    const DevModel &M = *a.model;
    if (a.op == OBJ_SET_STATE) {
        set_state(M, P, a.x, a.time);
    } else if (a.op == OBJ_STEP) {
        step(M, P, a.u, a.dt);
    } else if (a.op == OBJ_FORECAST) {
        set_state(M, P, a.x, a.time);
        const double zero[FR_C] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // Control::Zero()
        for (int64_t k = 0; k < a.steps; k++) {
            double *o = a.out + k * MPPI_DF_N;
            for (int i = 0; i < FR_NB; i++) o[MPPI_DF_JOINT_POSITION + i] = P.q[i];
            for (int i = 0; i < MPPI_EE_N; i++) o[MPPI_DF_END_EFFECTOR + i] = P.ee[i];
            o[MPPI_DF_JOINT_POWER] = 0.0;      // PinocchioDynamics::get_joint_power (.hpp:211-214)
            o[MPPI_DF_EXTERNAL_POWER] = 0.0;   // get_external_power (.hpp:220-223)
            o[MPPI_DF_ENERGY] = P.energy;
            for (int i = 0; i < 6; i++) o[MPPI_DF_WRENCH + i] = a.wrench ? a.wrench[k * 6 + i] : 0.0;
            step(M, P, zero, a.dt);   // add_end_effector_simulated_wrench is a no-op (.hpp:276)
        }
    } else if (a.op == OBJ_COST) {
        // get_cost(state, control, dynamics, time): the state's q / qd, the object's cached
        // kinematics (the lag of the reference's calculate()), its tank energy and its own state's
        // yaw (workspace / reach terms read dynamics->get_state()[2])
        double r[FR_NREC];
        for (int i = 0; i < FR_NB; i++) {
            r[REC_QQD + 2 * i] = a.x[i];
            r[REC_QQD + 2 * i + 1] = a.x[FR_NB + i];
        }
        for (int k = 0; k < 3; k++) {
            r[REC_EE + k] = P.ee[MPPI_EE_POSITION + k];
            r[REC_AM + k] = P.am[k];
            r[REC_VL + k] = P.ee[MPPI_EE_LINEAR_VELOCITY + k];
        }
        r[REC_E] = P.energy;
        r[REC_E + 1] = 0.0;
        const double *J = P.ee + MPPI_EE_JACOBIAN;   // J_a J_a^T, J_a = rows 0..2, arm columns 3..9
        int n = 0;
        for (int i = 0; i < 3; i++)
            for (int j = i; j < 3; j++, n++) {
                double s = 0.0;
                for (int c = FR_ARM0; c < FR_ARM1; c++) s += J[i * FR_NB + c] * J[j * FR_NB + c];
                r[REC_JJ + n] = s;
            }
        r[FR_NREC - 1] = 0.0;
        double t[7] = {0, 0, 0, 0, 0, 0, 0}, cost;
        if (a.cost.kind == MPPI_COST_TRACK_POINT) {
            cost = mppi_cost::track_point_cost(a.cost, r, P.state[2]);
        } else {
            mppi_cost::assisted_manipulation_terms(a.cost, a.sc, r, P.state[2], t);
            cost = 0.0;   // get_cost's running sum, term order (assisted_manipulation.cpp:48-71)
            for (int k = 0; k < 7; k++) cost += t[k];
        }
        a.out[0] = cost;
        for (int k = 0; k < 7; k++) a.out[1 + k] = t[k];
    }
}

namespace mppi_eng {

hipError_t launch_fr_object(const ObjArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(fr_object_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace mppi_eng
