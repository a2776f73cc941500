// mppi_oracle.cpp — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from
// the product (assistedmanipulation_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may use it, and only as the checker / the CPU baseline.
//
// A dependency-free fp64 restatement of the reference's MPPI hot path
// (LuigiVan01/AssistedManipulation @ 2025-02-05, paths relative to its src/):
//
//   controller/mppi.cpp            Trajectory::{create,update,sample,rollout,optimise,filter,get}
//   controller/gaussian.hpp        Gaussian (transform + mt19937/normal_distribution, or injected)
//   controller/filter.{hpp,cpp}    MovingExtendedWindow / SavitzkyGolayFilter
//   controller/gram_savitzky_golay GramPoly / GenFact / Weight / ComputeWeights
//   controller/cost.hpp            QuadraticCost, Left/RightInverseBarrierFunction
//   controller/energy.hpp          EnergyTank
//   frankaridgeback/pinocchio_dynamics.cpp:142-260   set_state / calculate / step
//   frankaridgeback/objective/assisted_manipulation.cpp:24-319   reset / get_cost / terms
//
// Pinocchio (v2.7.1, not vendored) is restated from its published algorithms: RNEA for
// nonLinearEffects, the articulated-body algorithm (aba), first-order forward kinematics,
// updateFramePlacements, computeFrameJacobian(WORLD), getFrameVelocity(WORLD).  Its parity is
// pinned by tests/golden (an independent numpy CRBA/finite-difference model), because the
// reference cannot be built here (Eigen3 + Pinocchio absent).
//
// The rigid-body + cost code is templated on the scalar so the same restatement can run in
// float (to measure fp32 sensitivity) and with a FLOP-counting scalar (algorithmic FLOPs).
// Compiled with -ffp-contract=off so results do not depend on FMA contraction.

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../include/mppi_amd.h"
#include "../include/mppi_amd_frankaridgeback.h"

namespace orc {

// ------------------------------------------------------------------------------------------
// FLOP-counting scalar (add/sub/mul/div/sqrt/transcendental = 1 each).
// ------------------------------------------------------------------------------------------
struct FlopCount {
    static thread_local uint64_t flops;
    // per-phase attribution for the executed-vs-algorithmic table (oracle_count_flops_phases):
    // mark(p) charges the FLOPs since the last mark to phase `last` and makes p the current one
    static thread_local uint64_t phase[8], at;
    static thread_local int last;
    static void mark(int p)
    {
        phase[last] += flops - at;
        at = flops;
        last = p;
    }
};
thread_local uint64_t FlopCount::flops = 0;
thread_local uint64_t FlopCount::phase[8] = {0, 0, 0, 0, 0, 0, 0, 0};
thread_local uint64_t FlopCount::at = 0;
thread_local int FlopCount::last = 0;

struct CF {
    double v;
    CF() : v(0) {}
    CF(double x) : v(x) {}
    explicit operator double() const { return v; }
};
inline CF operator+(CF a, CF b) { FlopCount::flops++; return CF(a.v + b.v); }
inline CF operator-(CF a, CF b) { FlopCount::flops++; return CF(a.v - b.v); }
inline CF operator*(CF a, CF b) { FlopCount::flops++; return CF(a.v * b.v); }
inline CF operator/(CF a, CF b) { FlopCount::flops++; return CF(a.v / b.v); }
inline CF operator-(CF a) { return CF(-a.v); }
inline CF &operator+=(CF &a, CF b) { a = a + b; return a; }
inline CF &operator-=(CF &a, CF b) { a = a - b; return a; }
inline CF &operator*=(CF &a, CF b) { a = a * b; return a; }
inline bool operator<(CF a, CF b) { return a.v < b.v; }
inline bool operator>(CF a, CF b) { return a.v > b.v; }
inline bool operator<=(CF a, CF b) { return a.v <= b.v; }
inline bool operator>=(CF a, CF b) { return a.v >= b.v; }

template <class T> inline T s_sin(T x) { return std::sin(x); }
template <class T> inline T s_cos(T x) { return std::cos(x); }
template <class T> inline T s_sqrt(T x) { return std::sqrt(x); }
template <class T> inline T s_acos(T x) { return std::acos(x); }
template <class T> inline T s_exp(T x) { return std::exp(x); }
template <class T> inline T s_fabs(T x) { return std::fabs(x); }
template <class T> inline bool s_isnan(T x) { return std::isnan(x); }
template <class T> inline T s_copysign(T a, T b) { return std::copysign(a, b); }
template <> inline CF s_sin(CF x) { FlopCount::flops++; return CF(std::sin(x.v)); }
template <> inline CF s_cos(CF x) { FlopCount::flops++; return CF(std::cos(x.v)); }
template <> inline CF s_sqrt(CF x) { FlopCount::flops++; return CF(std::sqrt(x.v)); }
template <> inline CF s_acos(CF x) { FlopCount::flops++; return CF(std::acos(x.v)); }
template <> inline CF s_exp(CF x) { FlopCount::flops++; return CF(std::exp(x.v)); }
template <> inline CF s_fabs(CF x) { return CF(std::fabs(x.v)); }
template <> inline bool s_isnan(CF x) { return std::isnan(x.v); }
template <> inline CF s_copysign(CF a, CF b) { return CF(std::copysign(a.v, b.v)); }
template <class T> inline T s_min(T a, T b) { return (b < a) ? b : a; }   // std::min
template <class T> inline T s_max(T a, T b) { return (a < b) ? b : a; }   // std::max
template <class T> inline double dbl(T x) { return (double)x; }

// ------------------------------------------------------------------------------------------
// Spatial algebra, Pinocchio conventions: a motion/force 6-vector is (linear, angular); an
// SE3 (R, p) maps child coordinates to parent coordinates.
// ------------------------------------------------------------------------------------------
template <class T> struct V3 {
    T x[3];
    V3() { x[0] = x[1] = x[2] = T(0); }
    V3(T a, T b, T c) { x[0] = a; x[1] = b; x[2] = c; }
    T &operator[](int i) { return x[i]; }
    const T &operator[](int i) const { return x[i]; }
};
template <class T> inline V3<T> operator+(const V3<T> &a, const V3<T> &b) { return V3<T>(a[0] + b[0], a[1] + b[1], a[2] + b[2]); }
template <class T> inline V3<T> operator-(const V3<T> &a, const V3<T> &b) { return V3<T>(a[0] - b[0], a[1] - b[1], a[2] - b[2]); }
template <class T> inline V3<T> operator*(T s, const V3<T> &a) { return V3<T>(s * a[0], s * a[1], s * a[2]); }
template <class T> inline V3<T> neg(const V3<T> &a) { return V3<T>(-a[0], -a[1], -a[2]); }
template <class T> inline T dot(const V3<T> &a, const V3<T> &b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
template <class T> inline V3<T> cross(const V3<T> &a, const V3<T> &b)
{
    return V3<T>(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
template <class T> inline T norm(const V3<T> &a) { return s_sqrt(dot(a, a)); }

template <class T> struct M3 {
    T a[9];   // row-major
    M3() { for (int i = 0; i < 9; i++) a[i] = T(0); }
    static M3 eye() { M3 m; m.a[0] = m.a[4] = m.a[8] = T(1); return m; }
    T &operator()(int r, int c) { return a[3 * r + c]; }
    const T &operator()(int r, int c) const { return a[3 * r + c]; }
};
template <class T> inline V3<T> mul(const M3<T> &m, const V3<T> &v)
{
    V3<T> r;
    for (int i = 0; i < 3; i++) r[i] = (m(i, 0) * v[0] + m(i, 1) * v[1]) + m(i, 2) * v[2];
    return r;
}
template <class T> inline V3<T> mulT(const M3<T> &m, const V3<T> &v)
{
    V3<T> r;
    for (int i = 0; i < 3; i++) r[i] = (m(0, i) * v[0] + m(1, i) * v[1]) + m(2, i) * v[2];
    return r;
}
template <class T> inline M3<T> mul(const M3<T> &a, const M3<T> &b)
{
    M3<T> r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r(i, j) = (a(i, 0) * b(0, j) + a(i, 1) * b(1, j)) + a(i, 2) * b(2, j);
    return r;
}

template <class T> struct SE3 {
    M3<T> R;
    V3<T> p;
    SE3() : R(M3<T>::eye()), p() {}
};
template <class T> inline SE3<T> compose(const SE3<T> &a, const SE3<T> &b)   // SE3::operator*
{
    SE3<T> r;
    r.R = mul(a.R, b.R);
    r.p = a.p + mul(a.R, b.p);
    return r;
}

template <class T> struct Motion { V3<T> v, w; };
template <class T> struct Force { V3<T> f, n; };

template <class T> inline Motion<T> act(const SE3<T> &M, const Motion<T> &m)   // SE3::act(Motion)
{
    Motion<T> r;
    r.w = mul(M.R, m.w);
    r.v = mul(M.R, m.v) + cross(M.p, r.w);
    return r;
}
template <class T> inline Motion<T> actInv(const SE3<T> &M, const Motion<T> &m)   // SE3::actInv(Motion)
{
    Motion<T> r;
    r.w = mulT(M.R, m.w);
    r.v = mulT(M.R, m.v - cross(M.p, m.w));
    return r;
}
template <class T> inline Force<T> act(const SE3<T> &M, const Force<T> &f)   // SE3::act(Force)
{
    Force<T> r;
    r.f = mul(M.R, f.f);
    r.n = mul(M.R, f.n) + cross(M.p, r.f);
    return r;
}
template <class T> inline Motion<T> mcross(const Motion<T> &a, const Motion<T> &b)   // a ^ b
{
    Motion<T> r;
    r.v = cross(a.w, b.v) + cross(a.v, b.w);
    r.w = cross(a.w, b.w);
    return r;
}
template <class T> inline Force<T> fcross(const Motion<T> &a, const Force<T> &f)   // a ^ f
{
    Force<T> r;
    r.f = cross(a.w, f.f);
    r.n = cross(a.w, f.n) + cross(a.v, f.f);
    return r;
}

template <class T> struct M6 {
    T a[36];
    M6() { for (int i = 0; i < 36; i++) a[i] = T(0); }
    T &operator()(int r, int c) { return a[6 * r + c]; }
    const T &operator()(int r, int c) const { return a[6 * r + c]; }
};
template <class T> inline void to6(const Motion<T> &m, T *x) { for (int i = 0; i < 3; i++) { x[i] = m.v[i]; x[3 + i] = m.w[i]; } }
template <class T> inline void to6(const Force<T> &m, T *x) { for (int i = 0; i < 3; i++) { x[i] = m.f[i]; x[3 + i] = m.n[i]; } }
template <class T> inline Force<T> mulF(const M6<T> &A, const Motion<T> &m)
{
    T x[6], y[6];
    to6(m, x);
    for (int i = 0; i < 6; i++) {
        T s = A(i, 0) * x[0];
        for (int j = 1; j < 6; j++) s += A(i, j) * x[j];
        y[i] = s;
    }
    Force<T> f;
    for (int i = 0; i < 3; i++) { f.f[i] = y[i]; f.n[i] = y[3 + i]; }
    return f;
}
// Y_parent = X^* Y X^{-1} with X^* = [[R, 0], [p^R, R]] (SE3actOn, aba.hxx)
template <class T> inline M6<T> se3ActOn(const SE3<T> &M, const M6<T> &Y)
{
    M6<T> A;   // force transform
    M3<T> px;
    px(0, 1) = -M.p[2]; px(0, 2) = M.p[1]; px(1, 0) = M.p[2]; px(1, 2) = -M.p[0]; px(2, 0) = -M.p[1]; px(2, 1) = M.p[0];
    M3<T> pR = mul(px, M.R);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            A(i, j) = M.R(i, j);
            A(3 + i, 3 + j) = M.R(i, j);
            A(3 + i, j) = pR(i, j);
        }
    M6<T> AY, R;
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            T s = A(i, 0) * Y(0, j);
            for (int k = 1; k < 6; k++) s += A(i, k) * Y(k, j);
            AY(i, j) = s;
        }
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            T s = AY(i, 0) * A(j, 0);
            for (int k = 1; k < 6; k++) s += AY(i, k) * A(j, k);
            R(i, j) = s;
        }
    return R;
}

// ------------------------------------------------------------------------------------------
// Model (from the mppi_frankaridgeback_desc table).
// ------------------------------------------------------------------------------------------
template <class T> struct Body {
    int parent;
    int type;
    V3<T> axis;
    SE3<T> placement;
    T mass;
    V3<T> lever;
    M3<T> Ic;
    M6<T> Y;   // spatial inertia matrix in the joint frame
};

template <class T> struct Model {
    int nb = 0;
    Body<T> b[MPPI_MAX_BODIES];
    int ee_parent = 0, am_parent = 0;
    SE3<T> ee_place, am_place;
    V3<T> gravity;
    int ee_support[MPPI_MAX_BODIES];   // 1 if body j supports the EE body

    void load(const mppi_frankaridgeback_desc &d)
    {
        nb = d.nbodies;
        for (int i = 0; i < nb; i++) {
            const mppi_body &s = d.bodies[i];
            Body<T> &o = b[i];
            o.parent = s.parent;
            o.type = s.type;
            o.axis = V3<T>(T(s.axis[0]), T(s.axis[1]), T(s.axis[2]));
            for (int k = 0; k < 9; k++) o.placement.R.a[k] = T(s.rotation[k]);
            o.placement.p = V3<T>(T(s.translation[0]), T(s.translation[1]), T(s.translation[2]));
            o.mass = T(s.mass);
            o.lever = V3<T>(T(s.lever[0]), T(s.lever[1]), T(s.lever[2]));
            // Symmetric3 order xx, xy, yy, xz, yz, zz
            const double *I = s.inertia;
            o.Ic(0, 0) = T(I[0]); o.Ic(0, 1) = o.Ic(1, 0) = T(I[1]); o.Ic(1, 1) = T(I[2]);
            o.Ic(0, 2) = o.Ic(2, 0) = T(I[3]); o.Ic(1, 2) = o.Ic(2, 1) = T(I[4]); o.Ic(2, 2) = T(I[5]);
            // Inertia::matrix(): [[m E, -m[c]x], [m[c]x, Ic - m[c]x[c]x]]
            M6<T> Y;
            T m = o.mass;
            const V3<T> &c = o.lever;
            M3<T> cx;
            cx(0, 1) = -c[2]; cx(0, 2) = c[1]; cx(1, 0) = c[2]; cx(1, 2) = -c[0]; cx(2, 0) = -c[1]; cx(2, 1) = c[0];
            M3<T> cxcx = mul(cx, cx);
            for (int r = 0; r < 3; r++)
                for (int q = 0; q < 3; q++) {
                    Y(r, q) = (r == q) ? m : T(0);
                    Y(r, 3 + q) = -(m * cx(r, q));
                    Y(3 + r, q) = m * cx(r, q);
                    Y(3 + r, 3 + q) = o.Ic(r, q) - m * cxcx(r, q);
                }
            o.Y = Y;
        }
        ee_parent = d.end_effector.parent;
        am_parent = d.arm_mount.parent;
        for (int k = 0; k < 9; k++) { ee_place.R.a[k] = T(d.end_effector.rotation[k]); am_place.R.a[k] = T(d.arm_mount.rotation[k]); }
        ee_place.p = V3<T>(T(d.end_effector.translation[0]), T(d.end_effector.translation[1]), T(d.end_effector.translation[2]));
        am_place.p = V3<T>(T(d.arm_mount.translation[0]), T(d.arm_mount.translation[1]), T(d.arm_mount.translation[2]));
        gravity = V3<T>(T(d.gravity[0]), T(d.gravity[1]), T(d.gravity[2]));
        for (int j = 0; j < nb; j++) ee_support[j] = 0;
        for (int j = ee_parent; j >= 0; j = b[j].parent) ee_support[j] = 1;
    }

    // Joint model calc: placement of the joint's child frame relative to its joint frame
    // (JointModelR{X,Y,Z}/RevoluteUnaligned/P*/PrismaticUnaligned), and motion subspace S.
    SE3<T> jointM(int i, T q) const
    {
        SE3<T> M;
        const Body<T> &o = b[i];
        if (o.type == MPPI_JOINT_PRISMATIC) {
            M.p = q * o.axis;
        } else {
            // AngleAxis(q, axis).toRotationMatrix()  (Eigen; exact Rz for axis z)
            T s = s_sin(q), c = s_cos(q);
            const V3<T> &a = o.axis;
            if (dbl(a[0]) == 0.0 && dbl(a[1]) == 0.0 && dbl(a[2]) == 1.0) {   // JointModelRZ
                M.R(0, 0) = c; M.R(0, 1) = -s; M.R(1, 0) = s; M.R(1, 1) = c; M.R(2, 2) = T(1);
            } else {
                V3<T> sa = s * a;
                V3<T> c1a = (T(1) - c) * a;
                M.R(0, 1) = c1a[0] * a[1] - sa[2]; M.R(1, 0) = c1a[0] * a[1] + sa[2];
                M.R(0, 2) = c1a[0] * a[2] + sa[1]; M.R(2, 0) = c1a[0] * a[2] - sa[1];
                M.R(1, 2) = c1a[1] * a[2] - sa[0]; M.R(2, 1) = c1a[1] * a[2] + sa[0];
                M.R(0, 0) = c1a[0] * a[0] + c; M.R(1, 1) = c1a[1] * a[1] + c; M.R(2, 2) = c1a[2] * a[2] + c;
            }
        }
        return M;
    }
    Motion<T> S(int i) const
    {
        Motion<T> m;
        if (b[i].type == MPPI_JOINT_PRISMATIC) m.v = b[i].axis;
        else m.w = b[i].axis;
        return m;
    }
};

template <class T> inline T sdotS(const Motion<T> &S, const Force<T> &f) { return dot(S.v, f.f) + dot(S.w, f.n); }
template <class T> inline T Sdot6(const Motion<T> &S, const T *x) { return (S.v[0] * x[0] + S.v[1] * x[1] + S.v[2] * x[2]) + (S.w[0] * x[3] + S.w[1] * x[4] + S.w[2] * x[5]); }

// Kinematic/dynamic workspace (pinocchio::Data subset).
template <class T> struct Data {
    SE3<T> liMi[MPPI_MAX_BODIES], oMi[MPPI_MAX_BODIES];
    Motion<T> v[MPPI_MAX_BODIES], a[MPPI_MAX_BODIES];
    Force<T> f[MPPI_MAX_BODIES];
    M6<T> Yaba[MPPI_MAX_BODIES];
};

// pinocchio::nonLinearEffects (rnea.hxx, ddq = 0): tau = C(q,v) v + g(q)
template <class T> void nle(const Model<T> &M, Data<T> &D, const T *q, const T *qd, T *tau)
{
    Motion<T> a0;
    a0.v = neg(M.gravity);   // data.a_gf[0] = -model.gravity
    for (int i = 0; i < M.nb; i++) {
        const int p = M.b[i].parent;
        D.liMi[i] = compose(M.b[i].placement, M.jointM(i, q[i]));
        Motion<T> S = M.S(i);
        Motion<T> vj;
        vj.v = qd[i] * S.v;
        vj.w = qd[i] * S.w;
        D.v[i] = vj;
        if (p >= 0) {
            Motion<T> t = actInv(D.liMi[i], D.v[p]);
            D.v[i].v = D.v[i].v + t.v;
            D.v[i].w = D.v[i].w + t.w;
        }
        D.a[i] = mcross(D.v[i], vj);
        Motion<T> t = actInv(D.liMi[i], p >= 0 ? D.a[p] : a0);
        D.a[i].v = D.a[i].v + t.v;
        D.a[i].w = D.a[i].w + t.w;
        Force<T> Ya = mulF(M.b[i].Y, D.a[i]);
        Force<T> Yv = mulF(M.b[i].Y, D.v[i]);
        Force<T> vxYv = fcross(D.v[i], Yv);
        D.f[i].f = Ya.f + vxYv.f;
        D.f[i].n = Ya.n + vxYv.n;
    }
    for (int i = M.nb - 1; i >= 0; i--) {
        tau[i] = sdotS(M.S(i), D.f[i]);
        const int p = M.b[i].parent;
        if (p >= 0) {
            Force<T> t = act(D.liMi[i], D.f[i]);
            D.f[p].f = D.f[p].f + t.f;
            D.f[p].n = D.f[p].n + t.n;
        }
    }
}

// pinocchio::aba (aba.hxx, v2.x): articulated-body algorithm with velocity and gravity terms.
template <class T> void aba(const Model<T> &M, Data<T> &D, const T *q, const T *qd, const T *tau, T *ddq)
{
    T u[MPPI_MAX_BODIES];
    T Dinv[MPPI_MAX_BODIES];
    T UDinv[MPPI_MAX_BODIES][6];
    for (int i = 0; i < M.nb; i++) u[i] = tau[i];
    for (int i = 0; i < M.nb; i++) {   // AbaForwardStep1
        const int p = M.b[i].parent;
        D.liMi[i] = compose(M.b[i].placement, M.jointM(i, q[i]));
        Motion<T> S = M.S(i);
        Motion<T> vj;
        vj.v = qd[i] * S.v;
        vj.w = qd[i] * S.w;
        D.v[i] = vj;
        if (p >= 0) {
            Motion<T> t = actInv(D.liMi[i], D.v[p]);
            D.v[i].v = D.v[i].v + t.v;
            D.v[i].w = D.v[i].w + t.w;
        }
        D.a[i] = mcross(D.v[i], vj);
        D.Yaba[i] = M.b[i].Y;
        Force<T> Yv = mulF(M.b[i].Y, D.v[i]);
        D.f[i] = fcross(D.v[i], Yv);   // vxiv
    }
    for (int i = M.nb - 1; i >= 0; i--) {   // AbaBackwardStep
        const int p = M.b[i].parent;
        M6<T> &Ia = D.Yaba[i];
        Motion<T> S = M.S(i);
        T s6[6];
        to6(S, s6);
        T U[6];
        for (int r = 0; r < 6; r++) {
            T acc = Ia(r, 0) * s6[0];
            for (int c = 1; c < 6; c++) acc += Ia(r, c) * s6[c];
            U[r] = acc;
        }
        T Dd = Sdot6(S, U);
        Dinv[i] = T(1) / Dd;
        for (int r = 0; r < 6; r++) UDinv[i][r] = U[r] * Dinv[i];
        if (p >= 0)
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 6; c++) Ia(r, c) -= UDinv[i][r] * U[c];
        u[i] -= sdotS(S, D.f[i]);
        if (p >= 0) {
            Force<T> pa = D.f[i];
            Force<T> Iaa = mulF(Ia, D.a[i]);
            for (int k = 0; k < 3; k++) {
                pa.f[k] = pa.f[k] + (Iaa.f[k] + UDinv[i][k] * u[i]);
                pa.n[k] = pa.n[k] + (Iaa.n[k] + UDinv[i][3 + k] * u[i]);
            }
            M6<T> Yp = se3ActOn(D.liMi[i], Ia);
            for (int k = 0; k < 36; k++) D.Yaba[p].a[k] += Yp.a[k];
            Force<T> t = act(D.liMi[i], pa);
            D.f[p].f = D.f[p].f + t.f;
            D.f[p].n = D.f[p].n + t.n;
        }
    }
    Motion<T> a0;
    a0.v = neg(M.gravity);
    for (int i = 0; i < M.nb; i++) {   // AbaForwardStep2
        const int p = M.b[i].parent;
        Motion<T> t = actInv(D.liMi[i], p >= 0 ? D.a[p] : a0);
        D.a[i].v = D.a[i].v + t.v;
        D.a[i].w = D.a[i].w + t.w;
        T a6[6];
        to6(D.a[i], a6);
        T s = UDinv[i][0] * a6[0];
        for (int k = 1; k < 6; k++) s += UDinv[i][k] * a6[k];
        ddq[i] = Dinv[i] * u[i] - s;
        Motion<T> S = M.S(i);
        D.a[i].v = D.a[i].v + ddq[i] * S.v;
        D.a[i].w = D.a[i].w + ddq[i] * S.w;
    }
}

// ------------------------------------------------------------------------------------------
// FrankaRidgeback::PinocchioDynamics restated (pinocchio_dynamics.cpp:142-260).
// ------------------------------------------------------------------------------------------
template <class T> struct FrankaDynamics {
    const Model<T> *M = nullptr;
    Data<T> D;
    bool reduced = false;       // true: a = M^-1 tau_u with no NLE (minimal arithmetic)
    T q[12], qd[12], tau[12], qdd[12];
    T energy = T(0);
    T state[MPPI_FR_STATE];
    // cached kinematics (computed in calculate() BEFORE integration: the one-step lag)
    V3<T> ee_pos, am_pos, ee_lin_vel, ee_ang_vel;
    V3<T> ee_lin_acc, ee_ang_acc;   // getFrameAcceleration(WORLD) (:211-223)
    M3<T> ee_rot;                   // oMf[EE].rotation() (:217)
    T J[6][12];
    T power = T(0);

    void init(const Model<T> *m)
    {
        M = m;
        for (int i = 0; i < 12; i++) q[i] = qd[i] = tau[i] = qdd[i] = T(0);
        for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = T(0);
    }

    void set_state(const double *x)
    {
        for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = T(x[i]);
        for (int i = 0; i < 12; i++) { q[i] = state[i]; qd[i] = state[12 + i]; }
        energy = state[30];   // EnergyTank::set_energy
        calculate();
    }

    void calculate()
    {
        if (!reduced) {
            T n[12];
            nle(*M, D, q, qd, n);
            for (int i = 0; i < 12; i++) tau[i] += n[i];   // m_joint_torque += NLE (:156)
            aba(*M, D, q, qd, tau, qdd);
        } else {
            calculate_reduced();
            return;
        }
        // forwardKinematics(q, v, a) — placements, velocities and accelerations (Pinocchio's
        // forward pass, local frames: a_i = iXp a_p + S qdd + v_i x (S qd), no gravity)
        for (int i = 0; i < M->nb; i++) {
            const int p = M->b[i].parent;
            D.liMi[i] = compose(M->b[i].placement, M->jointM(i, q[i]));
            D.oMi[i] = p >= 0 ? compose(D.oMi[p], D.liMi[i]) : D.liMi[i];
            Motion<T> S = M->S(i);
            Motion<T> vj;
            vj.v = qd[i] * S.v;
            vj.w = qd[i] * S.w;
            D.v[i] = vj;
            D.a[i].v = qdd[i] * S.v;
            D.a[i].w = qdd[i] * S.w;
            if (p >= 0) {
                Motion<T> t = actInv(D.liMi[i], D.v[p]);
                D.v[i].v = D.v[i].v + t.v;
                D.v[i].w = D.v[i].w + t.w;
                Motion<T> ta = actInv(D.liMi[i], D.a[p]);
                Motion<T> c = mcross(D.v[i], vj);
                D.a[i].v = (ta.v + D.a[i].v) + c.v;
                D.a[i].w = (ta.w + D.a[i].w) + c.w;
            }
        }
        // updateFramePlacements: oMf = oMi[parent] * placement
        SE3<T> ee = compose(D.oMi[M->ee_parent], M->ee_place);
        SE3<T> am = compose(D.oMi[M->am_parent], M->am_place);
        ee_pos = ee.p;
        am_pos = am.p;
        // computeFrameJacobian(WORLD): column j = oMi[j].act(S_j) for j supporting the EE
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 12; c++) J[r][c] = T(0);
        for (int j = 0; j < M->nb; j++) {
            if (!M->ee_support[j]) continue;
            Motion<T> col = act(D.oMi[j], M->S(j));
            for (int k = 0; k < 3; k++) { J[k][j] = col.v[k]; J[3 + k][j] = col.w[k]; }
        }
        T yaw = q[2];   // top-left 3x3 overwritten with R_z(yaw) (:196-200)
        T cy = s_cos(yaw), sy = s_sin(yaw);
        J[0][0] = cy; J[0][1] = -sy; J[0][2] = T(0);
        J[1][0] = sy; J[1][1] = cy; J[1][2] = T(0);
        J[2][0] = T(0); J[2][1] = T(0); J[2][2] = T(1);
        // getFrameVelocity(WORLD) = oMi[parent].act(v[parent])
        Motion<T> vw = act(D.oMi[M->ee_parent], D.v[M->ee_parent]);
        ee_lin_vel = vw.v;
        ee_ang_vel = vw.w;
        Motion<T> aw = act(D.oMi[M->ee_parent], D.a[M->ee_parent]);   // getFrameAcceleration(WORLD)
        ee_lin_acc = aw.v;
        ee_ang_acc = aw.w;
        ee_rot = ee.R;
    }

    // Minimal arithmetic (used for FLOP counting and to bound the arithmetic difference):
    // a = M(q)^-1 tau_u by a zero-velocity, zero-gravity articulated-body pass carried out in
    // world coordinates (no parent/child inertia transforms), which equals the reference's
    // aba(q, v, tau_u + nle(q, v)) in exact arithmetic (pinocchio_dynamics.cpp:156-171).  The
    // world motion subspaces are the WORLD Jacobian columns; the frame velocity is J v.
    // phases of the executed-vs-algorithmic table: 0 FK and motion subspaces, 1 world
    // inertias, 2 the solve (articulated-body passes), 3 kinematics for the cost (EE / arm-mount
    // positions, J v, J), 4 integration (base velocity, Euler, tank), 5 the objective (get_cost)
    static void phase(int p)
    {
        if constexpr (std::is_same<T, CF>::value) FlopCount::mark(p);
        (void)p;
    }
    void calculate_reduced()
    {
        const int nb = M->nb;
        phase(0);
        V3<T> Sv[MPPI_MAX_BODIES], Sw[MPPI_MAX_BODIES];
        for (int i = 0; i < nb; i++) {
            const int p = M->b[i].parent;
            D.liMi[i] = compose(M->b[i].placement, M->jointM(i, q[i]));
            D.oMi[i] = p >= 0 ? compose(D.oMi[p], D.liMi[i]) : D.liMi[i];
            V3<T> ax = mul(D.oMi[i].R, M->b[i].axis);
            if (M->b[i].type == MPPI_JOINT_PRISMATIC) { Sv[i] = ax; Sw[i] = V3<T>(); }
            else { Sw[i] = ax; Sv[i] = cross(D.oMi[i].p, ax); }
        }
        phase(1);
        // symmetric 6x6 articulated inertias, world frame, packed upper triangle (21)
        T Ia[MPPI_MAX_BODIES][21];
        T pA[MPPI_MAX_BODIES][6];
        for (int i = 0; i < nb; i++) {
            const Body<T> &bd = M->b[i];
            const M3<T> &R = D.oMi[i].R;
            V3<T> c = mul(R, bd.lever) + D.oMi[i].p;
            M3<T> RI = mul(R, bd.Ic), Iw;
            for (int r = 0; r < 3; r++)
                for (int cc = r; cc < 3; cc++) Iw(r, cc) = (RI(r, 0) * R(cc, 0) + RI(r, 1) * R(cc, 1)) + RI(r, 2) * R(cc, 2);
            T m = bd.mass;
            V3<T> mc = m * c;
            // [[mE, -m[c]x], [m[c]x, Iw - m[c]x[c]x]] ; -[c]x[c]x = |c|^2 E - c c^T
            T cc2 = dot(c, c);
            T *P = Ia[i];
            int k = 0;
            T full[6][6];
            for (int r = 0; r < 3; r++) for (int q2 = 0; q2 < 3; q2++) full[r][q2] = (r == q2) ? m : T(0);
            full[0][3] = T(0); full[0][4] = mc[2]; full[0][5] = -mc[1];
            full[1][3] = -mc[2]; full[1][4] = T(0); full[1][5] = mc[0];
            full[2][3] = mc[1]; full[2][4] = -mc[0]; full[2][5] = T(0);
            for (int r = 0; r < 3; r++)
                for (int q2 = r; q2 < 3; q2++)
                    full[3 + r][3 + q2] = (r == q2) ? Iw(r, q2) + (m * cc2 - mc[r] * c[q2]) : Iw(r, q2) - mc[r] * c[q2];
            for (int r = 0; r < 6; r++)
                for (int q2 = r; q2 < 6; q2++) P[k++] = full[r][q2];
            for (int j = 0; j < 6; j++) pA[i][j] = T(0);
        }
        phase(2);
        auto idx = [](int r, int c) { if (r > c) { int t = r; r = c; c = t; } return r * 6 - r * (r - 1) / 2 + (c - r); };
        T U[MPPI_MAX_BODIES][6], Dinv[MPPI_MAX_BODIES], uu[MPPI_MAX_BODIES];
        for (int i = nb - 1; i >= 0; i--) {
            T s6[6] = {Sv[i][0], Sv[i][1], Sv[i][2], Sw[i][0], Sw[i][1], Sw[i][2]};
            for (int r = 0; r < 6; r++) {
                T acc = Ia[i][idx(r, 0)] * s6[0];
                for (int c2 = 1; c2 < 6; c2++) acc += Ia[i][idx(r, c2)] * s6[c2];
                U[i][r] = acc;
            }
            T Dd = s6[0] * U[i][0];
            for (int r = 1; r < 6; r++) Dd += s6[r] * U[i][r];
            Dinv[i] = T(1) / Dd;
            T sp = s6[0] * pA[i][0];
            for (int r = 1; r < 6; r++) sp += s6[r] * pA[i][r];
            uu[i] = tau[i] - sp;
            const int p = M->b[i].parent;
            if (p >= 0) {
                T ud = uu[i] * Dinv[i];
                int k = 0;
                for (int r = 0; r < 6; r++) {
                    T Ud = U[i][r] * Dinv[i];
                    for (int c2 = r; c2 < 6; c2++, k++) Ia[p][k] += Ia[i][k] - Ud * U[i][c2];
                }
                for (int r = 0; r < 6; r++) pA[p][r] += pA[i][r] + U[i][r] * ud;
            }
        }
        T acc6[MPPI_MAX_BODIES][6];
        for (int i = 0; i < nb; i++) {
            const int p = M->b[i].parent;
            T a6[6];
            for (int r = 0; r < 6; r++) a6[r] = p >= 0 ? acc6[p][r] : T(0);
            T ua = U[i][0] * a6[0];
            for (int r = 1; r < 6; r++) ua += U[i][r] * a6[r];
            qdd[i] = Dinv[i] * (uu[i] - ua);
            T s6[6] = {Sv[i][0], Sv[i][1], Sv[i][2], Sw[i][0], Sw[i][1], Sw[i][2]};
            for (int r = 0; r < 6; r++) acc6[i][r] = a6[r] + s6[r] * qdd[i];
        }
        phase(3);
        SE3<T> ee = compose(D.oMi[M->ee_parent], M->ee_place);
        SE3<T> am = compose(D.oMi[M->am_parent], M->am_place);
        ee_pos = ee.p;
        am_pos = am.p;
        for (int r = 0; r < 6; r++)
            for (int c2 = 0; c2 < 12; c2++) J[r][c2] = T(0);
        V3<T> vl, vw;
        bool first = true;
        for (int j = 0; j < nb; j++) {
            if (!M->ee_support[j]) continue;
            for (int k = 0; k < 3; k++) { J[k][j] = Sv[j][k]; J[3 + k][j] = Sw[j][k]; }
            if (first) { vl = qd[j] * Sv[j]; vw = qd[j] * Sw[j]; first = false; }
            else { vl = vl + qd[j] * Sv[j]; vw = vw + qd[j] * Sw[j]; }
        }
        T yaw = q[2];
        T cy = s_cos(yaw), sy = s_sin(yaw);
        J[0][0] = cy; J[0][1] = -sy; J[0][2] = T(0);
        J[1][0] = sy; J[1][1] = cy; J[1][2] = T(0);
        J[2][0] = T(0); J[2][1] = T(0); J[2][2] = T(1);
        ee_lin_vel = vl;
        ee_ang_vel = vw;
        phase(4);
    }

    const T *step(const T *u, T dt)
    {
        phase(4);
        T yaw = q[2];
        T c = s_cos(yaw), s = s_sin(yaw);   // Eigen::Rotation2Dd(yaw) * base_velocity
        qd[0] = c * u[0] + (-s) * u[1];
        qd[1] = s * u[0] + c * u[1];
        qd[2] = u[2];
        for (int i = 0; i < 12; i++) tau[i] = T(0);
        for (int i = 3; i < 10; i++) tau[i] = u[i];   // arm torques; gripper controls ignored
        calculate();
        for (int i = 0; i < 12; i++) qd[i] = qd[i] + qdd[i] * dt;   // semi-implicit Euler
        for (int i = 0; i < 12; i++) q[i] = q[i] + qd[i] * dt;
        power = tau[0] * qd[0];
        for (int i = 1; i < 12; i++) power += tau[i] * qd[i];
        energy = s_max(T(0), energy + power * dt);   // EnergyTank::step
        state[30] = energy;
        for (int i = 0; i < 12; i++) { state[i] = q[i]; state[12 + i] = qd[i]; }
        return state;
    }
};

// ------------------------------------------------------------------------------------------
// Cost primitives (controller/cost.hpp) and AssistedManipulation (assisted_manipulation.cpp).
// ------------------------------------------------------------------------------------------
template <class T> inline T quad(const mppi_quadratic &q, T v)
{
    return (T(q.constant_cost) + T(q.linear_cost) * s_fabs(v)) + T(q.quadratic_cost) * v * v;
}
template <class T> inline T right_barrier(const mppi_barrier &b, T v)
{
    if (v >= T(b.bound)) { T d = v - T(b.bound); return T(b.maximum_cost) + T(b.scale) * (d * d); }
    return s_min(T(b.scale) / (T(b.bound) - v), T(b.maximum_cost));
}
template <class T> inline T left_barrier(const mppi_barrier &b, T v)
{
    if (v <= T(b.bound)) { T d = T(b.bound) - v; return T(b.maximum_cost) + T(b.scale) * (d * d); }
    return s_min(T(b.scale) / (v - T(b.bound)), T(b.maximum_cost));
}

struct CostTerms { double joint, self_collision, workspace, energy, velocity, trajectory, manipulability; };

template <class T> struct AssistedManipulation {
    mppi_assisted_manipulation_desc cfg;
    const double *forecast = nullptr;   // [H][6] table, row k = wrench at t0 + k dt
    int64_t forecast_rows = 0;
    double t0 = 0.0, dt = 0.01;
    CostTerms acc{};

    void reset(double time) { t0 = time; acc = CostTerms{}; }

    T joint_limit(const T *x)
    {
        T cost = T(0);
        for (int i = 0; i < 12; i++) {
            T c = left_barrier(cfg.lower_joint_limit[i], x[i]) + right_barrier(cfg.upper_joint_limit[i], x[i]);
            cost += c;
        }
        return cost;
    }

    // get_link_position() is the zero stub for PinocchioDynamics (pinocchio_dynamics.hpp:189-192)
    T self_collision()
    {
        static const int pairs[20][2] = {{3, 6}, {3, 7}, {3, 8}, {3, 9}, {3, 10}, {4, 6}, {4, 7}, {4, 8},
            {4, 9}, {4, 10}, {5, 7}, {5, 8}, {5, 9}, {5, 10}, {6, 8}, {6, 9}, {6, 10}, {7, 9}, {7, 10}, {8, 10}};
        // Link enum: PIVOT=3, PANDA_LINK1..7 = 4..10 (dynamics.hpp Link); radii index = link - 3
        T cost = T(0);
        for (int k = 0; k < 20; k++) {
            T distance = norm(V3<T>() - V3<T>());
            T radii = T(cfg.self_collision_radii[pairs[k][0] - 3]) + T(cfg.self_collision_radii[pairs[k][1] - 3]);
            cost += left_barrier(cfg.self_collision_limit, distance - radii);
        }
        return cost;
    }

    T workspace(const FrankaDynamics<T> &d)
    {
        T cost = T(0);
        V3<T> ee = d.ee_pos;
        T ang = d.state[2];   // dynamics->get_state()[2]
        // AngleAxisd(ang, UnitZ).toRotationMatrix()
        T s = s_sin(ang), c = s_cos(ang);
        T r22 = (T(1) - c) + c;
        V3<T> forward(c, s, T(0));
        V3<T> off(T(0.1) * c + (-s) * T(0) + T(0) * T(0.15), T(0.1) * s + c * T(0) + T(0) * T(0.15),
                  T(0) * T(0.1) + T(0) * T(0) + r22 * T(0.15));
        V3<T> robot = d.am_pos + off;
        V3<T> to_ee = ee - robot;
        T projection = dot(to_ee, forward) / dot(forward, forward);
        cost += left_barrier(cfg.workspace_limit_infront, projection);
        T reach = norm(to_ee);
        cost += right_barrier(cfg.workspace_limit_reach, reach);
        T n1 = s_sqrt(to_ee[0] * to_ee[0] + to_ee[1] * to_ee[1]);
        T n2 = s_sqrt(forward[0] * forward[0] + forward[1] * forward[1]);
        T yaw = s_acos((to_ee[0] * forward[0] + to_ee[1] * forward[1]) / n1 / n2);
        if (!s_isnan(yaw)) cost += quad(cfg.workspace_cost_yaw, s_fabs(yaw));
        T height = ee[2] - robot[2];
        cost += left_barrier(cfg.workspace_limit_above, height);
        return cost;
    }

    T energy_term(const FrankaDynamics<T> &d)
    {
        return left_barrier(cfg.energy_limit_below, d.energy) + right_barrier(cfg.energy_limit_above, d.energy);
    }

    T velocity(const T *x)
    {
        T cost = T(0);
        for (int i = 0; i < 12; i++) {
            T v = s_fabs(x[12 + i]);
            cost += T(cfg.velocity_cost[i].quadratic_cost) * (v * v);
        }
        return cost;
    }

    T trajectory(const FrankaDynamics<T> &d, int64_t step)
    {
        if (!cfg.has_forecast) return T(0);
        V3<T> force;
        if (forecast && step < forecast_rows)
            force = V3<T>(T(forecast[6 * step + 0]), T(forecast[6 * step + 1]), T(forecast[6 * step + 2]));
        T mx = T(cfg.trajectory_target_maximum);
        V3<T> target;
        for (int k = 0; k < 3; k++) target[k] = s_max(s_min(T(cfg.trajectory_target_scale) * force[k], mx), -mx);
        T distance = norm(target);
        T cost = T(0);
        if (distance > T(cfg.trajectory_position_threshold)) {
            cost += quad(cfg.trajectory_position_cost, distance);
            T projection = dot(d.ee_lin_vel, target) / dot(target, target);
            projection = s_copysign(T(1), projection) * norm(projection * target);
            T vt = s_exp(T(cfg.trajectory_velocity_dropoff) * distance) - T(1);
            vt = std::clamp(vt, T(cfg.trajectory_velocity_minimum), T(cfg.trajectory_velocity_maximum));
            T err = s_fabs(vt - projection);
            cost += quad(cfg.trajectory_velocity_cost, err);
        }
        return cost;
    }

    T manipulability(const FrankaDynamics<T> &d)
    {
        // J.rightCols(12 - 3).topLeftCorner(3, 7) = rows 0..2, columns 3..9
        T m[3][3];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                T s = d.J[r][3] * d.J[c][3];
                for (int k = 4; k < 10; k++) s += d.J[r][k] * d.J[c][k];
                m[r][c] = s;
            }
        // Eigen 3x3 determinant (bruteforce_det3_helper)
        auto h = [&](int a, int b, int c) { return m[0][a] * (m[1][b] * m[2][c] - m[1][c] * m[2][b]); };
        T det = (h(0, 1, 2) - h(1, 0, 2)) + h(2, 0, 1);
        T volume = s_sqrt(det);
        if (s_isnan(volume)) volume = T(1e-5);
        else volume = std::clamp(volume, T(1e-5), T(1e5));
        return quad(cfg.manipulability_cost, T(1) / volume);
    }

    // get_cost (assisted_manipulation.cpp:37-72): terms in the reference's order.
    T get_cost(const T *x, const FrankaDynamics<T> &d, int64_t step)
    {
        T cost = T(0);
        if (cfg.enable_joint_limit) { T c = joint_limit(x); acc.joint += dbl(c); cost += c; }
        if (cfg.enable_self_collision_limit) { T c = self_collision(); acc.self_collision += dbl(c); cost += c; }
        if (cfg.enable_workspace_limit) { T c = workspace(d); acc.workspace += dbl(c); cost += c; }
        if (cfg.enable_energy_limit) { T c = energy_term(d); acc.energy += dbl(c); cost += c; }
        if (cfg.enable_velocity_cost) { T c = velocity(x); acc.velocity += dbl(c); cost += c; }
        if (cfg.enable_trajectory_cost) { T c = trajectory(d, step); acc.trajectory += dbl(c); cost += c; }
        if (cfg.enable_manipulability_cost) { T c = manipulability(d); acc.manipulability += dbl(c); cost += c; }
        return cost;
    }
};

// ------------------------------------------------------------------------------------------
// TrackPoint (frankaridgeback/objective/track_point.cpp:10-186), SURVEY §8f item 1.
// ------------------------------------------------------------------------------------------
template <class T> struct TrackPoint {
    mppi_track_point_desc cfg;

    void reset(double) {}

    // point_cost (:36-43): 100 pow(|p_EE - point|, 2)
    T point(const FrankaDynamics<T> &d)
    {
        T distance = norm(d.ee_pos - V3<T>(T(cfg.point[0]), T(cfg.point[1]), T(cfg.point[2])));
        return T(100.0) * (distance * distance);
    }

    // joint_limit_cost (:45-95): static limits, joints 0..9
    T joint_limit(const T *x)
    {
        static const double lower[12] = {-2.0, -2.0, -6.28, -2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973, 0.5, 0.5};
        static const double upper[12] = {2.0, 2.0, 6.28, 2.8973, 1.7628, 2.8973, 0.0698, 2.8973, 3.7525, 2.8973, 0.5, 0.5};
        T cost = T(0);
        for (int i = 0; i < 10; i++) {
            if (x[i] < T(lower[i])) { T dd = T(lower[i]) - x[i]; cost += T(1000.0) + T(100000.0) * (dd * dd); }
            if (x[i] > T(upper[i])) { T dd = x[i] - T(upper[i]); cost += T(1000.0) + T(100000.0) * (dd * dd); }
        }
        return cost;
    }

    // self_collision_cost (:97-160) with get_link_position == 0; collision = radii - distance
    T self_collision()
    {
        static const int pairs[20][2] = {{3, 6}, {3, 7}, {3, 8}, {3, 9}, {3, 10}, {4, 6}, {4, 7}, {4, 8},
            {4, 9}, {4, 10}, {5, 7}, {5, 8}, {5, 9}, {5, 10}, {6, 8}, {6, 9}, {6, 10}, {7, 9}, {7, 10}, {8, 10}};
        T cost = T(0);
        for (int k = 0; k < 20; k++) {
            T distance = norm(V3<T>() - V3<T>());
            T radii = T(cfg.self_collision_radii[pairs[k][0] - 3]) + T(cfg.self_collision_radii[pairs[k][1] - 3]);
            cost += left_barrier(cfg.self_collision_limit, radii - distance);
        }
        return cost;
    }

    // reach_cost (:162-186)
    T reach(const FrankaDynamics<T> &d)
    {
        T ang = d.state[2];
        T s = s_sin(ang), c = s_cos(ang);
        T r22 = (T(1) - c) + c;
        V3<T> off(T(0.3) * c + (-s) * T(0) + T(0) * T(0.15), T(0.3) * s + c * T(0) + T(0) * T(0.15),
                  T(0) * T(0.3) + T(0) * T(0) + r22 * T(0.15));
        V3<T> robot = d.am_pos + off;
        return right_barrier(cfg.maximum_reach_limit, norm(d.ee_pos - robot));
    }

    // get_cost (:10-34)
    T get_cost(const T *x, const FrankaDynamics<T> &d, int64_t)
    {
        T cost = point(d);
        if (cfg.enable_joint_limits) cost += joint_limit(x);
        if (cfg.enable_self_collision_avoidance) cost += self_collision();
        if (cfg.enable_reach_limits) cost += reach(d);
        return cost;
    }
};

// ------------------------------------------------------------------------------------------
// Point-mass bring-up plugin (not in the reference).  State (p, v), control
// force; semi-implicit Euler as in a8; cost sum q (p - p*)^2 + r u^2.
// ------------------------------------------------------------------------------------------
struct PointMass {
    double mass = 1.0;
    double state[6];
    void set_state(const double *x) { for (int i = 0; i < 6; i++) state[i] = x[i]; }
    const double *step(const double *u, double dt)
    {
        for (int i = 0; i < 3; i++) state[3 + i] = state[3 + i] + (u[i] / mass) * dt;
        for (int i = 0; i < 3; i++) state[i] = state[i] + state[3 + i] * dt;
        return state;
    }
};
inline double point_cost(const mppi_quadratic_cost_desc &c, const double *x, const double *u)
{
    double cost = 0.0;
    for (int i = 0; i < 3; i++) { double d = x[i] - c.target[i]; cost += c.q[i] * (d * d); }
    for (int i = 0; i < 3; i++) cost += c.r[i] * (u[i] * u[i]);
    return cost;
}

// ------------------------------------------------------------------------------------------
// Savitzky-Golay (gram_savitzky_golay.cpp, filter.cpp) restated.
// ------------------------------------------------------------------------------------------
static double GramPoly(int i, int m, int k, int s)
{
    if (k > 0)
        return (4. * k - 2.) / (k * (2. * m - k + 1.)) * (i * GramPoly(i, m, k - 1, s) + s * GramPoly(i, m, k - 1, s - 1)) -
               ((k - 1.) * (2. * m + k)) / (k * (2. * m - k + 1.)) * GramPoly(i, m, k - 2, s);
    return (k == 0 && s == 0) ? 1. : 0.;
}
static double GenFact(int a, int b)
{
    double gf = 1.;
    for (int j = (a - b) + 1; j <= a; j++) gf *= j;
    return gf;
}
static double SGWeight(int i, int t, int m, int n, int s)
{
    double w = 0;
    for (int k = 0; k <= n; ++k)
        w = w + (2 * k + 1) * (GenFact(2 * m, k) / GenFact(2 * m + k + 1, k + 1)) * GramPoly(i, m, k, 0) * GramPoly(t, m, k, s);
    return w;
}
static std::vector<double> SGWeights(int m, int t, int n, int s)
{
    std::vector<double> w(2 * (size_t)m + 1);
    for (int i = 0; i < 2 * m + 1; ++i) w[(size_t)i] = SGWeight(i - m, t, m, n, s);
    return w;
}

struct MovingExtendedWindow {
    int window;
    double last_trim_t;
    size_t start_idx;
    std::vector<double> uu, tt;
    MovingExtendedWindow(int size, int w) : window(w), last_trim_t(-1), start_idx((size_t)w)
    {
        uu.assign((size_t)size + 2 * (size_t)window + 1, 0.0);
        tt.assign((size_t)size + 2 * (size_t)window + 1, -1.0);
    }
    void trim(double t)
    {
        if (t < last_trim_t) throw std::runtime_error("Resetting the window back in the past.");
        last_trim_t = t;
        size_t trim_idx = start_idx;
        for (size_t i = 0; i < start_idx; i++)
            if (tt[i] >= t) { trim_idx = i; break; }
        size_t offset = trim_idx - (size_t)window;
        std::rotate(tt.begin(), tt.begin() + (long)offset, tt.end());
        std::rotate(uu.begin(), uu.begin() + (long)offset, uu.end());
        if (offset > 0) {
            std::fill(tt.end() - (long)offset, tt.end(), *(tt.end() - (long)offset - 1));
            std::fill(uu.end() - (long)offset, uu.end(), *(uu.end() - (long)offset - 1));
        }
        start_idx = (size_t)window;
        tt[start_idx] = t;
    }
    void add_point(double u, double t)
    {
        if (t < tt[start_idx]) throw std::runtime_error("Adding measurement older then new time");
        uu[start_idx] = u;
        tt[start_idx] = t;
        std::fill(uu.begin() + (long)start_idx + 1, uu.end(), uu[start_idx]);
        std::fill(tt.begin() + (long)start_idx + 1, tt.end(), tt[start_idx]);
        start_idx++;
    }
    size_t lower(double t) const { return (size_t)std::distance(tt.begin(), std::lower_bound(tt.begin(), tt.end(), t)); }
    void set(double u, double t) { uu[lower(t) - 1] = u; }
};

struct SGFilter {
    std::vector<double> weights;
    std::vector<MovingExtendedWindow> windows;
    SGFilter(int steps, int nu, int window, int order)
    {
        weights = SGWeights(window, 0, order, 0);
        windows.assign((size_t)nu, MovingExtendedWindow(steps, window));
    }
    void reset(double t) { for (auto &w : windows) w.trim(t); }
    void add_measurement(const double *u, double t) { for (size_t i = 0; i < windows.size(); i++) windows[i].add_point(u[i], t); }
    void apply(double *u, double t)
    {
        for (size_t i = 0; i < windows.size(); i++) {
            MovingExtendedWindow &w = windows[i];
            size_t idx = w.lower(t);
            double res = weights[0] * w.uu[idx - (size_t)w.window];
            for (size_t k = 1; k < weights.size(); ++k) res += weights[k] * w.uu[idx - (size_t)w.window + k];
            u[i] = res / 1.0;   // dt_ = pow(time_step = 1, 0)
            w.set(u[i], t);
        }
    }
};

// ------------------------------------------------------------------------------------------
// Simple persistent pool: contiguous-block partition of rollouts (mppi.cpp:272-307).
// ------------------------------------------------------------------------------------------
class Pool {
public:
    explicit Pool(unsigned n) : stop_(false), gen_(0), done_(0)
    {
        for (unsigned i = 1; i < n; i++) threads_.emplace_back([this, i] { loop(i); });
        n_ = n;
    }
    ~Pool()
    {
        { std::lock_guard<std::mutex> l(m_); stop_ = true; gen_++; }
        cv_.notify_all();
        for (auto &t : threads_) t.join();
    }
    void run(const std::function<void(unsigned)> &fn)
    {
        if (n_ == 1) { fn(0); return; }
        { std::lock_guard<std::mutex> l(m_); fn_ = &fn; done_ = 0; gen_++; }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> l(m_);
        dcv_.wait(l, [this] { return done_ == n_ - 1; });
    }
private:
    void loop(unsigned id)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)> *f;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = fn_;
            }
            (*f)(id);
            { std::lock_guard<std::mutex> l(m_); done_++; }
            dcv_.notify_one();
        }
    }
    std::vector<std::thread> threads_;
    std::mutex m_;
    std::condition_variable cv_, dcv_;
    bool stop_;
    uint64_t gen_;
    unsigned done_, n_ = 1;
    const std::function<void(unsigned)> *fn_ = nullptr;
};

// ------------------------------------------------------------------------------------------
// Symmetric eigendecomposition (cyclic Jacobi) for Gaussian::set_covariance: T = V sqrt(L).
// Eigen's SelfAdjointEigenSolver orders eigenvalues ascending; we do the same.  The exact
// column order/sign among ties is implementation-defined, which is why parity runs inject eps.
// ------------------------------------------------------------------------------------------
static void gaussian_transform(int n, const double *cov_colmajor, std::vector<double> &T)
{
    std::vector<double> A((size_t)n * n), V((size_t)n * n, 0.0);
    for (int c = 0; c < n; c++)
        for (int r = 0; r < n; r++) A[(size_t)r * n + c] = cov_colmajor[(size_t)c * n + r];
    for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) off += A[(size_t)p * n + q] * A[(size_t)p * n + q];
        if (off < 1e-30) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                double apq = A[(size_t)p * n + q];
                if (std::fabs(apq) < 1e-300) continue;
                double app = A[(size_t)p * n + p], aqq = A[(size_t)q * n + q];
                double theta = (aqq - app) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; k++) {
                    double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
                    A[(size_t)k * n + p] = c * akp - s * akq;
                    A[(size_t)k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
                    A[(size_t)p * n + k] = c * apk - s * aqk;
                    A[(size_t)q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
                    V[(size_t)k * n + p] = c * vkp - s * vkq;
                    V[(size_t)k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    std::vector<int> order((size_t)n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return A[(size_t)a * n + a] < A[(size_t)b * n + b]; });
    T.assign((size_t)n * n, 0.0);   // row-major n x n
    for (int j = 0; j < n; j++) {
        int src = order[(size_t)j];
        double l = std::max(0.0, A[(size_t)src * n + src]);
        for (int i = 0; i < n; i++) T[(size_t)i * n + j] = V[(size_t)i * n + src] * std::sqrt(l);
    }
}

// ------------------------------------------------------------------------------------------
// mppi::Trajectory restated (mppi.cpp).  Costs, weights, gradient and controls are fp64; the
// rollout's dynamics/cost run in Scalar (double = the reference; float = sensitivity probe).
// ------------------------------------------------------------------------------------------
struct Trajectory {
    mppi_config cfg{};
    mppi_dynamics_desc dyn{};
    mppi_cost_desc costd{};
    int scalar = 0;            // 0 double, 1 float
    int reduced = 0;           // 1: minimal arithmetic (zero-bias ABA, no NLE)
    int compat_uint8 = 0;
    int64_t S = 0, K = 0, R = 0, H = 0, C = 0, X = 0;
    double dt = 0;
    unsigned threads = 1;
    std::vector<double> init_state, cov, cmin, cmax, cdefault;
    bool has_default = false;
    std::vector<std::vector<double>> noise;   // [R][k*C + c]
    std::vector<double> cost, weights, gradient, U, Ushift, rollout_state;
    double optimal_cost = 0;
    double update_last = 0, update_duration = 0, rollout_time = 0, last_rollout_time = 0, last_shift_time = 0;
    int64_t shift_by = 0, shifted = 0;
    uint64_t update_count = 0;
    std::vector<double> forecast;   // H x 6
    Model<double> md;
    Model<float> mf;
    std::unique_ptr<SGFilter> sg;
    std::unique_ptr<Pool> pool;
    // noise source
    int injected = 1;
    std::vector<double> inj;        // pending eps columns
    size_t inj_pos = 0;
    std::mt19937 gen;
    std::normal_distribution<double> ndist{0.0, 1.0};
    std::vector<double> Tg;         // gaussian transform (row-major)
    std::string err;
    CostTerms optimal_terms{};
    // sharded mode (rehearses the engine's multi-GPU exchange): only rollouts [shard_begin,
    // shard_end) are rolled out, then `allreduce` sums the cost vector and the partial gradient.
    int64_t shard_begin = 0, shard_end = -1;
    void (*allreduce)(double *, int64_t) = nullptr;

    bool draw(double *out)
    {
        if (injected) {
            if (inj_pos + (size_t)C > inj.size()) return false;
            for (int64_t c = 0; c < C; c++) out[c] = inj[inj_pos + (size_t)c];
            inj_pos += (size_t)C;
            return true;
        }
        std::vector<double> z((size_t)C);   // VectorXd(m_mean.size()).unaryExpr(...)
        for (auto &v : z) v = ndist(gen);
        for (int64_t i = 0; i < C; i++) {
            double s = 0.0;
            for (int64_t j = 0; j < C; j++) s += Tg[(size_t)(i * C + j)] * z[(size_t)j];
            out[i] = 0.0 + s;
        }
        return true;
    }

    int64_t draws_needed(double time) const
    {
        int64_t sb = (int64_t)((time - last_shift_time) / dt);
        int64_t keep = keep_count();
        int64_t d = (S - keep) * H;
        if (sb > 0) d += keep * std::min<int64_t>(sb, H);
        return d;
    }
    int64_t keep_count() const { return compat_uint8 ? (int64_t)(uint8_t)K : K; }

    int sample(double time)
    {
        shift_by = (int64_t)((time - last_shift_time) / dt);
        if (shift_by > 0) {
            last_shift_time = time;
            shifted = std::max<int64_t>(0, H - shift_by);   // H - shift_by < 0 is UB in the reference
            for (int64_t k = 0; k < shifted; k++)
                for (int64_t c = 0; c < C; c++) Ushift[(size_t)(k * C + c)] = U[(size_t)((k + shift_by) * C + c)];
            for (int64_t k = shifted; k < H; k++)
                for (int64_t c = 0; c < C; c++) Ushift[(size_t)(k * C + c)] = U[(size_t)((H - 1) * C + c)];
        }
        std::vector<int64_t> order((size_t)S);
        std::iota(order.begin(), order.end(), 2);
        // mppi.cpp:225-231 sorts with `cost[l] < cost[r]`.  With a NaN cost that comparator is not a
        // strict weak order, so std::stable_sort's result is undefined; the defined reading used
        // here (and by the device) is: NaN costs sort after every number, ties keep index order.
        std::stable_sort(order.begin(), order.end(), [this](int64_t l, int64_t r) {
            const double a = cost[(size_t)l], b = cost[(size_t)r];
            if (std::isnan(a)) return false;
            if (std::isnan(b)) return true;
            return a < b;
        });
        int64_t keep = std::min<int64_t>(keep_count(), S);
        if (shift_by > 0) {
            for (int64_t p = 0; p < keep; p++) {
                std::vector<double> &n = noise[(size_t)order[(size_t)p]];
                for (int64_t k = 0; k < shifted; k++)
                    for (int64_t c = 0; c < C; c++) n[(size_t)(k * C + c)] = n[(size_t)((k + shift_by) * C + c)];
                for (int64_t k = shifted; k < H; k++)
                    if (!draw(&n[(size_t)(k * C)])) return MPPI_ERR_NOISE;
            }
        }
        for (int64_t p = keep; p < S; p++) {
            std::vector<double> &n = noise[(size_t)order[(size_t)p]];
            for (int64_t k = 0; k < H; k++)
                if (!draw(&n[(size_t)(k * C)])) return MPPI_ERR_NOISE;
        }
        for (int64_t i = 0; i < C * H; i++) noise[1][(size_t)i] = -U[(size_t)i];   // -m_optimal_control
        return MPPI_OK;
    }

    template <class T> double rollout_franka(const double *eps, bool optimal, CostTerms *terms, FrankaDynamics<T> &d)
    {
        const Model<T> *m;
        if constexpr (std::is_same<T, double>::value) m = &md;
        else m = &mf;
        if (d.M != m) d.init(m);
        d.reduced = reduced != 0;
        if (costd.kind == MPPI_COST_TRACK_POINT) {
            TrackPoint<T> c;
            c.cfg = costd.track_point;
            return rollout_franka_with(c, eps, optimal, d);
        }
        AssistedManipulation<T> c;
        c.cfg = costd.assisted_manipulation;
        c.forecast = forecast.empty() ? nullptr : forecast.data();
        c.forecast_rows = (int64_t)forecast.size() / 6;
        c.dt = dt;
        const double total = rollout_franka_with(c, eps, optimal, d);
        if (terms) *terms = c.acc;
        return total;
    }

    // rollout() (mppi.cpp:311-342) of one sample with objective c
    template <class T, class Obj> double rollout_franka_with(Obj &c, const double *eps, bool optimal, FrankaDynamics<T> &d)
    {
        d.set_state(rollout_state.data());
        c.reset(rollout_time);
        double total = 0.0;
        T state[MPPI_FR_STATE];
        for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = T(rollout_state[(size_t)i]);
        T u[MPPI_FR_CONTROL];
        for (int64_t k = 0; k < H; k++) {
            for (int64_t i = 0; i < C; i++)
                u[i] = T(eps ? Ushift[(size_t)(k * C + i)] + eps[k * C + i] : Ushift[(size_t)(k * C + i)]);
            double sc = std::pow(cfg.cost_discount_factor, (double)k) * dbl(c.get_cost(state, d, k));
            if (!optimal && std::isnan(sc)) { total = NAN; break; }
            total += sc;
            const T *x = d.step(u, T(dt));
            for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = x[i];
        }
        return total;
    }

    double rollout_point(const double *eps, bool optimal)
    {
        PointMass pm;
        pm.mass = dyn.point_mass.mass;
        pm.set_state(rollout_state.data());
        double state[6];
        for (int i = 0; i < 6; i++) state[i] = rollout_state[(size_t)i];
        double total = 0.0, u[3];
        for (int64_t k = 0; k < H; k++) {
            for (int i = 0; i < 3; i++) u[i] = eps ? Ushift[(size_t)(k * C + i)] + eps[k * C + i] : Ushift[(size_t)(k * C + i)];
            double sc = std::pow(cfg.cost_discount_factor, (double)k) * point_cost(costd.quadratic, state, u);
            if (!optimal && std::isnan(sc)) { total = NAN; break; }
            total += sc;
            const double *x = pm.step(u, dt);
            for (int i = 0; i < 6; i++) state[i] = x[i];
        }
        return total;
    }

    double rollout_one(const double *eps, bool optimal, CostTerms *terms, FrankaDynamics<double> &dd, FrankaDynamics<float> &df)
    {
        if (dyn.kind == MPPI_DYNAMICS_POINT_MASS) return rollout_point(eps, optimal);
        if (scalar == 1) return rollout_franka<float>(eps, optimal, terms, df);
        return rollout_franka<double>(eps, optimal, terms, dd);
    }

    std::vector<FrankaDynamics<double>> dyn_d;   // per-thread plugin copies (mppi.cpp:137-140)
    std::vector<FrankaDynamics<float>> dyn_f;

    void rollout()
    {
        const int64_t b0 = shard_begin, e0 = shard_end < 0 ? R : shard_end;
        const int64_t n = e0 - b0;
        int64_t each = n / (int64_t)threads, distribute = n % (int64_t)threads;
        std::vector<std::pair<int64_t, int64_t>> ranges;
        int64_t start = b0;
        for (unsigned t = 0; t < threads; t++) {
            int64_t stop = start + each;
            if (distribute > 0) { stop += 1; distribute -= 1; }
            if (start == stop) break;
            ranges.emplace_back(start, stop);
            start = stop;
        }
        if (shard_end >= 0)
            for (int64_t r = 0; r < R; r++)
                if (r < b0 || r >= e0) cost[(size_t)r] = 0.0;
        pool->run([&](unsigned t) {
            if (t >= ranges.size()) return;
            for (int64_t r = ranges[t].first; r < ranges[t].second; r++)
                cost[(size_t)r] = rollout_one(noise[(size_t)r].data(), false, nullptr, dyn_d[t], dyn_f[t]);
        });
        if (allreduce) allreduce(cost.data(), R);
    }

    int optimise()
    {
        int64_t valid = 0, imin = -1, imax = -1;
        for (int64_t i = 0; i < R; i++) {
            double c = cost[(size_t)i];
            if (std::isnan(c)) continue;
            valid++;
            if (imin < 0 || c < cost[(size_t)imin]) imin = i;       // first minimum
            if (imax < 0 || !(c < cost[(size_t)imax])) imax = i;    // last maximum
        }
        if (valid <= 1) { err = "all nan rollouts"; return MPPI_ERR_ALL_NAN; }
        double minimum = cost[(size_t)imin], maximum = cost[(size_t)imax];
        double difference = maximum - minimum;
        if (difference < 1e-6) return MPPI_OK;
        double total = 0.0;
        for (int64_t i = 0; i < R; i++) {
            double c = cost[(size_t)i];
            if (std::isnan(c)) { weights[(size_t)i] = 0.0; continue; }
            double l = std::exp(-cfg.cost_scale * (c - minimum) / difference);
            total += l;
            weights[(size_t)i] = l;
        }
        for (auto &w : weights) w = w / total;
        if (shard_end < 0) {
            for (int64_t j = 0; j < C * H; j++) gradient[(size_t)j] = noise[0][(size_t)j] * weights[0];
            for (int64_t i = 1; i < R; i++)
                for (int64_t j = 0; j < C * H; j++) gradient[(size_t)j] += noise[(size_t)i][(size_t)j] * weights[(size_t)i];
        } else {   // partial sum over the shard, then summed across shards
            for (int64_t j = 0; j < C * H; j++) gradient[(size_t)j] = 0.0;
            for (int64_t i = shard_begin; i < shard_end; i++)
                for (int64_t j = 0; j < C * H; j++) gradient[(size_t)j] += noise[(size_t)i][(size_t)j] * weights[(size_t)i];
            if (allreduce) allreduce(gradient.data(), C * H);
        }
        for (int64_t j = 0; j < C * H; j++) Ushift[(size_t)j] += gradient[(size_t)j] * cfg.gradient_step;
        if (sg) {
            try {
                sg->reset(rollout_time);
                for (int64_t k = 0; k < H; k++) sg->add_measurement(&Ushift[(size_t)(k * C)], rollout_time + (double)k * dt);
                for (int64_t k = 0; k < H; k++) sg->apply(&Ushift[(size_t)(k * C)], rollout_time + (double)k * dt);
            } catch (const std::exception &e) {
                err = e.what();
                return MPPI_ERR_SMOOTHING;
            }
        }
        if (cfg.control_bound)
            for (int64_t k = 0; k < H; k++)
                for (int64_t c = 0; c < C; c++) {
                    double &u = Ushift[(size_t)(k * C + c)];
                    u = std::max(std::min(u, cmax[(size_t)c]), cmin[(size_t)c]);
                }
        return MPPI_OK;
    }

    int update(const double *state, double time)
    {
        for (int64_t i = 0; i < X; i++) rollout_state[(size_t)i] = state[i];
        rollout_time = time;
        auto t0 = std::chrono::steady_clock::now();
        int st = sample(time);
        if (st != MPPI_OK) { err = "injected noise stream too short"; return st; }
        rollout();
        st = optimise();
        if (st != MPPI_OK) return st;
        optimal_cost = rollout_one(nullptr, true, &optimal_terms, dyn_d[0], dyn_f[0]);   // filter()
        last_rollout_time = rollout_time;
        U = Ushift;
        update_duration = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        update_last = time;
        ++update_count;
        if (injected) { inj.erase(inj.begin(), inj.begin() + (long)inj_pos); inj_pos = 0; }
        return MPPI_OK;
    }

    int get(double time, double *control)
    {
        if (time < last_rollout_time) return MPPI_ERR_TIME;
        double t = (time - last_rollout_time) / dt;
        int lower = (int)t, upper = lower + 1;
        if (upper >= H) {
            for (int64_t c = 0; c < C; c++)
                control[c] = has_default ? cdefault[(size_t)c] : U[(size_t)((H - 1) * C + c)];
            return MPPI_OK;
        }
        t -= lower;
        for (int64_t c = 0; c < C; c++)
            control[c] = (1.0 - t) * U[(size_t)(lower * C + c)] + t * U[(size_t)(upper * C + c)];
        return MPPI_OK;
    }
};

static thread_local std::string g_err;

}   // namespace orc

using orc::Trajectory;

extern "C" {

const char *oracle_last_error(void *h) { return h ? ((Trajectory *)h)->err.c_str() : orc::g_err.c_str(); }

// Trajectory::create validation (mppi.cpp:17-69) + construction (mppi.cpp:79-152).
void *oracle_create(const mppi_config *cfg, const mppi_dynamics_desc *dyn, const mppi_cost_desc *cost,
                    int scalar, int reduced, int compat_uint8)
{
    int64_t Cd = dyn->kind == MPPI_DYNAMICS_POINT_MASS ? 3 : MPPI_FR_CONTROL;
    int64_t Xd = dyn->kind == MPPI_DYNAMICS_POINT_MASS ? 6 : MPPI_FR_STATE;
    int64_t Cc = cost->kind == MPPI_COST_QUADRATIC ? 3 : MPPI_FR_CONTROL;   // AssistedManipulation, TrackPoint
    int64_t Xc = cost->kind == MPPI_COST_QUADRATIC ? 6 : MPPI_FR_STATE;
    auto fail = [](const char *m) -> void * { orc::g_err = m; return nullptr; };
    if (Cd != Cc) return fail("controller dynamics control dof != cost control dof");
    if (Xd != Xc) return fail("controller dynamics state dof != cost state dof");
    if (cfg->control_dof != Cd || cfg->state_dof != Xd) return fail("configuration dof mismatch");
    if (!cfg->control_min || !cfg->control_max) return fail("controller maximum and minimum must have length control dof");
    if (!cfg->covariance) return fail("controller covariance matrix not square");
    if (cfg->rollouts < 1) return fail("trajectory rollouts must be greater than zero");
    if (cfg->keep_best_rollouts < 0) return fail("trajectory cached rollouts cannot be less than zero");
    if (cfg->threads <= 0) return fail("trajectory threads must be positive nonzero");
    if (compat_uint8 && cfg->rollouts + 2 > 255) return fail("compat uint8 index semantics require rollouts + 2 <= 255");
    if (!compat_uint8 && cfg->keep_best_rollouts > cfg->rollouts) return fail("keep_best_rollouts > rollouts");
    Trajectory *t = new Trajectory();
    t->cfg = *cfg;
    t->dyn = *dyn;
    t->costd = *cost;
    t->scalar = scalar;
    t->reduced = reduced;
    t->compat_uint8 = compat_uint8;
    t->S = cfg->rollouts;
    t->K = cfg->keep_best_rollouts;
    t->R = t->S + 2;
    t->dt = cfg->time_step;
    t->H = (int64_t)std::ceil(cfg->horison / cfg->time_step);
    t->C = Cd;
    t->X = Xd;
    t->threads = cfg->threads;
    t->init_state.assign(cfg->initial_state, cfg->initial_state + Xd);
    t->cov.assign(cfg->covariance, cfg->covariance + Cd * Cd);
    t->cmin.assign(cfg->control_min, cfg->control_min + Cd);
    t->cmax.assign(cfg->control_max, cfg->control_max + Cd);
    t->has_default = cfg->has_control_default != 0;
    if (t->has_default) t->cdefault.assign(cfg->control_default, cfg->control_default + Cd);
    t->noise.assign((size_t)t->R, std::vector<double>((size_t)(t->C * t->H), 0.0));
    t->cost.assign((size_t)t->R, 0.0);
    t->weights.assign((size_t)t->R, 0.0);
    t->gradient.assign((size_t)(t->C * t->H), 0.0);
    t->U.assign((size_t)(t->C * t->H), 0.0);
    t->Ushift.assign((size_t)(t->C * t->H), 0.0);
    t->rollout_state.assign((size_t)Xd, 0.0);   // m_rollout_state.setZero() (mppi.cpp:121)
    if (dyn->kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        t->md.load(dyn->frankaridgeback);
        t->mf.load(dyn->frankaridgeback);
    }
    if (cfg->has_smoothing)
        t->sg.reset(new orc::SGFilter((int)t->H, (int)t->C, (int)cfg->smoothing_window, (int)cfg->smoothing_order));
    t->pool.reset(new orc::Pool(t->threads));
    t->dyn_d.resize(t->threads);
    t->dyn_f.resize(t->threads);
    orc::gaussian_transform((int)t->C, cfg->covariance, t->Tg);
    return t;
}

void oracle_destroy(void *h) { delete (Trajectory *)h; }

int oracle_set_noise_source(void *h, int injected, uint64_t seed)
{
    Trajectory *t = (Trajectory *)h;
    t->injected = injected;
    if (!injected) t->gen.seed((std::mt19937::result_type)seed);
    return MPPI_OK;
}
int oracle_inject_noise(void *h, const double *eps, int64_t columns)
{
    Trajectory *t = (Trajectory *)h;
    t->inj.insert(t->inj.end(), eps, eps + columns * t->C);
    return MPPI_OK;
}
int64_t oracle_noise_draws(void *h, double time) { return ((Trajectory *)h)->draws_needed(time); }
int oracle_set_forecast(void *h, const double *table)
{
    Trajectory *t = (Trajectory *)h;
    if (table) t->forecast.assign(table, table + 6 * t->H);
    else t->forecast.clear();
    return MPPI_OK;
}
int oracle_update(void *h, const double *state, double time)
{
    try {
        return ((Trajectory *)h)->update(state, time);
    } catch (const std::exception &e) {
        ((Trajectory *)h)->err = e.what();
        return MPPI_ERR_INVALID;
    }
}
int oracle_get(void *h, double time, double *control) { return ((Trajectory *)h)->get(time, control); }
void oracle_dims(void *h, int64_t *R, int64_t *H, int64_t *C, int64_t *X)
{
    Trajectory *t = (Trajectory *)h;
    *R = t->R; *H = t->H; *C = t->C; *X = t->X;
}
void oracle_costs(void *h, double *out) { Trajectory *t = (Trajectory *)h; std::copy(t->cost.begin(), t->cost.end(), out); }
// Test hook: the previous update's rollout costs, which the next sample() sorts (mppi.cpp:222-231).
// Used after an engine failure that has no reference counterpart (an in-launch wait timing out),
// so that the oracle's next update starts from the engine's state.
void oracle_set_costs(void *h, const double *in) { Trajectory *t = (Trajectory *)h; std::copy(in, in + t->R, t->cost.begin()); }
void oracle_weights(void *h, double *out) { Trajectory *t = (Trajectory *)h; std::copy(t->weights.begin(), t->weights.end(), out); }
void oracle_gradient(void *h, double *out) { Trajectory *t = (Trajectory *)h; std::copy(t->gradient.begin(), t->gradient.end(), out); }
void oracle_optimal_control(void *h, double *out) { Trajectory *t = (Trajectory *)h; std::copy(t->U.begin(), t->U.end(), out); }
double oracle_optimal_cost(void *h) { return ((Trajectory *)h)->optimal_cost; }
double oracle_update_duration(void *h) { return ((Trajectory *)h)->update_duration; }
void oracle_noise(void *h, double *out)
{
    Trajectory *t = (Trajectory *)h;
    for (int64_t r = 0; r < t->R; r++) std::copy(t->noise[(size_t)r].begin(), t->noise[(size_t)r].end(), out + r * t->C * t->H);
}
void oracle_set_threads(void *h, unsigned threads)
{
    Trajectory *t = (Trajectory *)h;
    t->threads = threads;
    t->pool.reset(new orc::Pool(threads));
    t->dyn_d.resize(threads);
    t->dyn_f.resize(threads);
}
void oracle_smoothing_windows(void *h, double *uu, double *tt, int64_t *start_idx)
{
    Trajectory *t = (Trajectory *)h;
    if (!t->sg) return;
    size_t o = 0;
    for (size_t c = 0; c < t->sg->windows.size(); c++) {
        const auto &w = t->sg->windows[c];
        std::copy(w.uu.begin(), w.uu.end(), uu + o);
        std::copy(w.tt.begin(), w.tt.end(), tt + o);
        start_idx[c] = (int64_t)w.start_idx;
        o += w.uu.size();
    }
}

void oracle_set_shard(void *h, int64_t begin, int64_t end, void (*allreduce)(double *, int64_t))
{
    Trajectory *t = (Trajectory *)h;
    t->shard_begin = begin;
    t->shard_end = end;
    t->allreduce = allreduce;
}

// Optimal rollout's per-term totals (BaseTest reads them by downcasting, base.cpp:141-146).
void oracle_optimal_terms(void *h, double *out7)
{
    const orc::CostTerms &c = ((Trajectory *)h)->optimal_terms;
    out7[0] = c.joint; out7[1] = c.self_collision; out7[2] = c.workspace; out7[3] = c.energy;
    out7[4] = c.velocity; out7[5] = c.trajectory; out7[6] = c.manipulability;
}


// ---- FrankaRidgeback::PinocchioDynamics as an object (the engine's mppi_dynamics_*) ----------
// pinocchio_dynamics.cpp:84-260 on the Pinocchio-order restatement above: the constructor's
// setZero()s and set_state, set_state / step / get_state / get_end_effector_state, and
// DynamicsForecast::forecast (frankaridgeback/dynamics.cpp:104-138).
struct OracleDyn {
    orc::Model<double> m;
    orc::FrankaDynamics<double> d;
    double time = 0.0;
};

// EndEffectorState in the engine's MPPI_EE_* layout (100 doubles); the quaternion by Eigen's
// Quaternion(Matrix3) (quaternionbase_assign_impl), coefficients (x, y, z, w)
static void oracle_ee_row(const orc::FrankaDynamics<double> &d, double *o)
{
    for (int k = 0; k < 3; k++) o[k] = d.ee_pos[k];
    const double *R = d.ee_rot.a;
    double q[4];
    const double t = R[0] + R[4] + R[8];
    if (t > 0.0) {
        double s = std::sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (R[7] - R[5]) * s;
        q[1] = (R[2] - R[6]) * s;
        q[2] = (R[3] - R[1]) * s;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (R[3 * k + j] - R[3 * j + k]) * s;
        q[j] = (R[3 * j + i] + R[3 * i + j]) * s;
        q[k] = (R[3 * k + i] + R[3 * i + k]) * s;
    }
    for (int k = 0; k < 4; k++) o[3 + k] = q[k];
    for (int k = 0; k < 9; k++) o[7 + k] = R[k];
    for (int k = 0; k < 3; k++) {
        o[16 + k] = d.ee_lin_vel[k];
        o[19 + k] = d.ee_ang_vel[k];
        o[22 + k] = d.ee_lin_acc[k];
        o[25 + k] = d.ee_ang_acc[k];
    }
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 12; c++) o[28 + 12 * r + c] = d.J[r][c];
}

void *oracle_dyn_create(const mppi_frankaridgeback_desc *desc, const double *x0)
{
    OracleDyn *o = new OracleDyn;
    o->m.load(*desc);
    o->d.init(&o->m);   // setZero()s (pinocchio_dynamics.cpp:106-109)
    o->d.set_state(x0);
    return o;
}

void oracle_dyn_destroy(void *h) { delete (OracleDyn *)h; }

void oracle_dyn_set_state(void *h, const double *x, double time)
{
    OracleDyn *o = (OracleDyn *)h;
    o->time = time;
    o->d.set_state(x);
}

void oracle_dyn_step(void *h, const double *u, double dt, double *x_out)
{
    OracleDyn *o = (OracleDyn *)h;
    const double *x = o->d.step(u, dt);
    o->time += dt;
    if (x_out)
        for (int i = 0; i < MPPI_FR_STATE; i++) x_out[i] = x[i];
}

void oracle_dyn_get_state(void *h, double *x)
{
    for (int i = 0; i < MPPI_FR_STATE; i++) x[i] = ((OracleDyn *)h)->d.state[i];
}

void oracle_dyn_end_effector(void *h, double *ee100) { oracle_ee_row(((OracleDyn *)h)->d, ee100); }

// q, v, a, tau (12 each), tank energy, power, time, arm-mount position (3): MPPI_DYNAMICS_QUERY_N
void oracle_dyn_query(void *h, double *out)
{
    const OracleDyn *o = (const OracleDyn *)h;
    const orc::FrankaDynamics<double> &d = o->d;
    for (int i = 0; i < 12; i++) {
        out[i] = d.q[i];
        out[12 + i] = d.qd[i];
        out[24 + i] = d.qdd[i];
        out[36 + i] = d.tau[i];
    }
    out[48] = d.energy;
    out[49] = d.power;
    out[50] = o->time;
    for (int k = 0; k < 3; k++) out[51 + k] = d.am_pos[k];
}

// DynamicsForecast::forecast (dynamics.cpp:104-138): rows of MPPI_DF_N (121) doubles
void oracle_dyn_forecast(void *h, const double *x, double time, double time_step, int64_t steps, const double *wrench,
                         double *out)
{
    OracleDyn *o = (OracleDyn *)h;
    oracle_dyn_set_state(h, x, time);
    const double zero[MPPI_FR_CONTROL] = {0};
    for (int64_t k = 0; k < steps; k++) {
        double *r = out + k * 121;
        for (int i = 0; i < 12; i++) r[i] = o->d.q[i];
        oracle_ee_row(o->d, r + 12);
        r[112] = 0.0;   // get_joint_power
        r[113] = 0.0;   // get_external_power
        r[114] = o->d.energy;
        for (int i = 0; i < 6; i++) r[115 + i] = wrench ? wrench[6 * k + i] : 0.0;
        oracle_dyn_step(h, zero, time_step, nullptr);
    }
}

// Cost::get_cost(state, control, dynamics, time) against the object (the engine's
// mppi_cost_evaluate): out8 = cost, seven AssistedManipulation terms (zeros for TrackPoint)
void oracle_cost_evaluate(const mppi_cost_desc *cost, void *h, const double *x, const double *wrench6, double *out8)
{
    OracleDyn *o = (OracleDyn *)h;
    for (int i = 0; i < 8; i++) out8[i] = 0.0;
    if (cost->kind == MPPI_COST_TRACK_POINT) {
        orc::TrackPoint<double> c;
        c.cfg = cost->track_point;
        out8[0] = c.get_cost(x, o->d, 0);
        return;
    }
    orc::AssistedManipulation<double> c;
    c.cfg = cost->assisted_manipulation;
    if (!wrench6) c.cfg.has_forecast = 0;   // no forecast handle: trajectory_cost is 0 (:239-240)
    c.forecast = wrench6;
    c.forecast_rows = wrench6 ? 1 : 0;
    c.reset(0.0);
    out8[0] = c.get_cost(x, o->d, 0);
    const orc::CostTerms &t = c.acc;
    out8[1] = t.joint; out8[2] = t.self_collision; out8[3] = t.workspace; out8[4] = t.energy;
    out8[5] = t.velocity; out8[6] = t.trajectory; out8[7] = t.manipulability;
}

// ---- per-step probes for the golden-vector tests ------------------------------------------
// calculate() at (q, v) with joint torque tau_u: outputs a (12), ee position (3), arm-mount
// position (3), frame Jacobian WORLD 6x12 row-major after the yaw overwrite (72), EE spatial
// velocity WORLD (6), NLE (12).  mode 0 = reference arithmetic, 1 = zero-bias ABA.
void oracle_kinematics(const mppi_frankaridgeback_desc *desc, const double *q, const double *v,
                       const double *tau_u, int mode, double *out)
{
    orc::Model<double> m;
    m.load(*desc);
    orc::FrankaDynamics<double> d;
    d.init(&m);
    d.reduced = mode == 1;
    for (int i = 0; i < 12; i++) { d.q[i] = q[i]; d.qd[i] = v[i]; d.tau[i] = tau_u[i]; }
    double n[12];
    orc::Data<double> D2;
    orc::nle(m, D2, q, v, n);
    d.calculate();
    int o = 0;
    for (int i = 0; i < 12; i++) out[o++] = d.qdd[i];
    for (int i = 0; i < 3; i++) out[o++] = d.ee_pos[i];
    for (int i = 0; i < 3; i++) out[o++] = d.am_pos[i];
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 12; c++) out[o++] = d.J[r][c];
    for (int i = 0; i < 3; i++) out[o++] = d.ee_lin_vel[i];
    for (int i = 0; i < 3; i++) out[o++] = d.ee_ang_vel[i];
    for (int i = 0; i < 12; i++) out[o++] = n[i];
    if (mode == 1) return;   // the minimal-arithmetic path forms no EE orientation / acceleration
    for (int i = 0; i < 9; i++) out[o++] = d.ee_rot.a[i];
    for (int i = 0; i < 3; i++) out[o++] = d.ee_lin_acc[i];
    for (int i = 0; i < 3; i++) out[o++] = d.ee_ang_acc[i];
}

// One rollout of FrankaRidgeback + AssistedManipulation from x0 with controls u (H x C,
// column-major) and forecast table; writes per-step cost (H) and the final state (31).
// scalar 0 = double, 1 = float; mode as above.
double oracle_rollout(const mppi_frankaridgeback_desc *desc, const mppi_assisted_manipulation_desc *cost,
                      const double *x0, const double *u, int64_t H, double dt, double t0,
                      const double *forecast, int scalar, int mode, double *step_costs, double *x_final)
{
    auto run = [&](auto tag) -> double {
        using T = decltype(tag);
        orc::Model<T> m;
        m.load(*desc);
        orc::FrankaDynamics<T> d;
        d.init(&m);
        d.reduced = mode == 1;
        orc::AssistedManipulation<T> c;
        c.cfg = *cost;
        c.forecast = forecast;
        c.forecast_rows = forecast ? H : 0;
        c.dt = dt;
        d.set_state(x0);
        c.reset(t0);
        T state[MPPI_FR_STATE];
        for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = T(x0[i]);
        double total = 0;
        for (int64_t k = 0; k < H; k++) {
            T uu[12];
            for (int i = 0; i < 12; i++) uu[i] = T(u[k * 12 + i]);
            double sc = orc::dbl(c.get_cost(state, d, k));
            if (step_costs) step_costs[k] = sc;
            total += sc;
            const T *x = d.step(uu, T(dt));
            for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = x[i];
        }
        if (x_final)
            for (int i = 0; i < MPPI_FR_STATE; i++) x_final[i] = orc::dbl(state[i]);
        return total;
    };
    if (scalar == 1) return run(float(0));
    return run(double(0));
}

// Algorithmic FLOPs of one rollout-step of the minimal arithmetic the device executes:
// zero-bias ABA (a = M^-1 tau_u) + kinematics/Jacobian/frame velocity + full default cost +
// integration.  Counted with a FLOP-counting scalar over `steps` steps from x0.
// cost_part (optional): the FLOPs of that total spent in get_cost (the device's cost kernel; the
// rest is the rollout kernel's FK, kinematics, ABA and integration).
double oracle_count_flops_split(const mppi_frankaridgeback_desc *desc, const mppi_assisted_manipulation_desc *cost,
                                const double *x0, int64_t steps, double *cost_part)
{
    orc::Model<orc::CF> m;
    m.load(*desc);
    orc::FrankaDynamics<orc::CF> d;
    d.init(&m);
    d.reduced = true;
    orc::AssistedManipulation<orc::CF> c;
    c.cfg = *cost;
    static double table[6 * 4096];
    for (int k = 0; k < 4096; k++) { table[6 * k] = 20.0; for (int j = 1; j < 6; j++) table[6 * k + j] = 0; }
    c.forecast = table;
    c.forecast_rows = 4096;
    d.set_state(x0);
    orc::CF state[MPPI_FR_STATE];
    for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = orc::CF(x0[i]);
    orc::FlopCount::flops = 0;
    for (auto &v : orc::FlopCount::phase) v = 0;   // (set_state's calculate() above is not counted)
    orc::FlopCount::at = 0;
    orc::FlopCount::last = 4;
    uint64_t in_cost = 0;
    for (int64_t k = 0; k < steps; k++) {
        orc::CF uu[12];
        for (int i = 0; i < 12; i++) uu[i] = orc::CF(0.1 * (double)((i * 7 + k) % 5 - 2));
        const uint64_t f0 = orc::FlopCount::flops;
        c.get_cost(state, d, k);
        in_cost += orc::FlopCount::flops - f0;
        const orc::CF *x = d.step(uu, orc::CF(0.01));
        for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = x[i];
    }
    if (cost_part) *cost_part = (double)in_cost / (double)steps;
    return (double)orc::FlopCount::flops / (double)steps;
}

// The same count split by phase (FrankaDynamics::phase: FK, world inertias, solve, kinematics,
// integration, objective), per rollout-step: out6[6].  Test / analysis infrastructure.
double oracle_count_flops_phases(const mppi_frankaridgeback_desc *desc, const mppi_assisted_manipulation_desc *cost,
                                 const double *x0, int64_t steps, double *out6)
{
    using orc::FlopCount;
    double cost_part = 0.0;
    // get_cost is phase 5: oracle_count_flops_split times it, the rest is marked inside the dynamics
    const double tot = oracle_count_flops_split(desc, cost, x0, steps, &cost_part);
    FlopCount::mark(4);
    // every get_cost ran inside phase 4 (between step()'s marks): move its FLOPs to phase 5
    FlopCount::phase[4] -= (uint64_t)(cost_part * (double)steps + 0.5);
    FlopCount::phase[5] = (uint64_t)(cost_part * (double)steps + 0.5);
    for (int p = 0; p < 6; p++) out6[p] = (double)FlopCount::phase[p] / (double)steps;
    return tot;
}

double oracle_count_flops(const mppi_frankaridgeback_desc *desc, const mppi_assisted_manipulation_desc *cost,
                          const double *x0, int64_t steps)
{
    return oracle_count_flops_split(desc, cost, x0, steps, nullptr);
}

// Savitzky-Golay weights (ComputeWeights(m, t, n, s)).
void oracle_sg_weights(int m, int t, int n, int s, double *out)
{
    std::vector<double> w = orc::SGWeights(m, t, n, s);
    std::copy(w.begin(), w.end(), out);
}

// Default descriptors from the generated model header.
void oracle_default_frankaridgeback(mppi_frankaridgeback_desc *d) { mppi_frankaridgeback_model(d); }
void oracle_default_assisted_manipulation(mppi_assisted_manipulation_desc *a) { mppi_assisted_manipulation_default(a); }

}   // extern "C"
