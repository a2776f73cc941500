// fr_cost_terms.hpp — the FrankaRidgeback objectives evaluated on one step record (kernels.hpp
// FR_REC stored layout, FR_NREC derived layout).  Shared by fr_step_cost_kernel (fr_cost.hip) and the rollout kernel's consumer
// waves (fr_coop.hip).
//
// AssistedManipulation::get_cost (assisted_manipulation.cpp:58-128) and TrackPoint::get_cost
// (frankaridgeback/objective/track_point.cpp:10-34), term order kept.  The joint-limit and
// velocity sums keep the association of the lane sums they replaced: (joints 0..5) + (6..11).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "fsincos.hpp"

namespace mppi_cost {

using namespace mppi_eng;
using mppi_dev::smin;

constexpr int CK_ASSISTED_MANIPULATION = 1, CK_TRACK_POINT = 3;   // mppi_cost_kind

// x / d from v_rcp_f64 and one Newton correction applied to the product (four ops; the rcp's
// 2.8e-8 relative error squares to ~1e-15, against the IEEE quotient's ten-op sequence).  Only
// for barrier quotients: d = 0 (v on the bound) gives NaN, and there the barrier selects `over`.
__device__ __forceinline__ double fquot(double x, double d)
{
    const double r = __builtin_amdgcn_rcp(d);
    const double t = x * r;
    const double e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(t, e, t);
}

// AssistedManipulation barriers (assisted_manipulation.cpp), written as selects
__device__ __forceinline__ double right_barrier(double bound, double scale, double mx, double v)
{
    const double d = v - bound;
    const double over = mx + scale * (d * d);
    const double under = smin(fquot(scale, bound - v), mx);
    return (v >= bound) ? over : under;
}
__device__ __forceinline__ double left_barrier(double bound, double scale, double mx, double v)
{
    const double d = bound - v;
    const double over = mx + scale * (d * d);
    const double under = smin(fquot(scale, v - bound), mx);
    return (v <= bound) ? over : under;
}
__device__ __forceinline__ double right_barrier(const DevBarrier &b, double v) { return right_barrier(b.bound, b.scale, b.max, v); }
__device__ __forceinline__ double left_barrier(const DevBarrier &b, double v) { return left_barrier(b.bound, b.scale, b.max, v); }

// Per-joint parameters of the objective in LDS, joint j at Lj[j JS ..]: lower barrier (bound,
// scale, max), upper barrier, velocity weight - uniform loads next to their use instead of 84
// scalar registers the compiler loaded up front and spilled.  fr_cost.hip stages them with stride
// JT_STRIDE; the rollout kernel reads them from its body table.
constexpr int JT_STRIDE = 7;

// trajectory_cost's velocity part on the EE frame velocity (assisted_manipulation.cpp:237-290)
__device__ __forceinline__ double trajectory_term(const DevCost &Cs, const StepConst &sc, const double *vl)
{
    double proj = ((vl[0] * sc.target[0] + vl[1] * sc.target[1]) + vl[2] * sc.target[2]) / sc.tt;
    const double p0 = proj * sc.target[0], p1 = proj * sc.target[1], p2 = proj * sc.target[2];
    proj = copysign(1.0, proj) * sqrt((p0 * p0 + p1 * p1) + p2 * p2);
    const double err = fabs(sc.vtarget - proj);
    const double tc = sc.pos_cost + ((Cs.traj_vel_c + Cs.traj_vel_l * fabs(err)) + Cs.traj_vel_q * err * err);
    return sc.active ? tc : 0.0;
}

// manipulability_cost on J_a J_a^T (assisted_manipulation.cpp:224-235)
__device__ __forceinline__ double manipulability_term(const DevCost &Cs, const double *jj)
{
    const double m00 = jj[0], m01 = jj[1], m02 = jj[2], m11 = jj[3], m12 = jj[4], m22 = jj[5];
    const double det = (m00 * (m11 * m22 - m12 * m12) - m01 * (m01 * m22 - m12 * m02)) + m02 * (m01 * m12 - m11 * m02);
    double vol = sqrt(det);
    vol = isnan(vol) ? 1e-5 : ((vol < 1e-5) ? 1e-5 : ((1e5 < vol) ? 1e5 : vol));
    const double iv = 1.0 / vol;
    return (Cs.manip_c + Cs.manip_l * fabs(iv)) + Cs.manip_q * iv * iv;
}

// J v and J_a J_a^T of a stored record (kernels.hpp REC_S01 / REC_S2Q) by the chains the rollout
// kernel's lanes ran before r05, term for term: lane m of a row summed over the bodies i = 0..9, in
// order, acc = fma(x_i, y_i, acc) from acc = 0, with x_i = S_i[m] and y_i = qd_i for J v (m < 3),
// and x_i = S_i[a], y_i = S_i[b] (y_i = 0 for the base, i < 3) for the packed J_a J_a^T entry (a, b)
// - so the sums, and every cost, keep their bits.
__device__ __forceinline__ void kin_sums(const double2 *rec2, double *vl, double *jj)
{
    double s0[10], s1[10], s2[10], qd[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const double2 a = rec2[REC_S01 / 2 + i], b = rec2[REC_S2Q / 2 + i];
        s0[i] = a.x;
        s1[i] = a.y;
        s2[i] = b.x;
        qd[i] = b.y;
    }
    const double *S[3] = {s0, s1, s2};
    constexpr int ja[6] = {0, 0, 0, 1, 1, 2}, jb[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
    for (int m = 0; m < 3; m++) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 10; i++) acc = __builtin_fma(S[m][i], qd[i], acc);
        vl[m] = acc;
    }
    // (the base's three terms of J_a J_a^T are fma(x, 0, +0) = +0 on the rows' chains, store_ks: a
    // chain that starts at body 3 from +0 has the same bits for finite S)
#pragma unroll
    for (int p = 0; p < 6; p++) {
        double acc = 0.0;
#pragma unroll
        for (int i = 3; i < 10; i++) acc = __builtin_fma(S[ja[p]][i], S[jb[p]][i], acc);
        jj[p] = acc;
    }
}

// The derived record (FR_NREC) of a stored one (FR_REC; a compact FR_REC_C record is one already)
__device__ __forceinline__ void derive_record(const double *rk, double *r, bool compact = false)
{
    const double2 *src = reinterpret_cast<const double2 *>(rk);
    const int n = compact ? FR_NREC / 2 : REC_VL / 2;
    for (int i = 0; i < n; i++) {
        const double2 v = src[i];
        r[2 * i] = v.x;
        r[2 * i + 1] = v.y;
    }
    if (!compact) kin_sums(src, r + REC_VL, r + REC_JJ);
    r[FR_NREC - 1] = 0.0;
}

// AssistedManipulation::get_cost at the record's state with its kinematics (KC: a compact record,
// J v and J_a J_a^T stored; else the 768-B record, whose motion subspaces they are formed from)
template <bool EN, int JS, bool KC = false, int JG = 1>
__device__ __forceinline__ double assisted_manipulation_cost(const DevCost &Cs, const StepConst &sc, const double *r,
                                                             const double *Lj, const double2 *src)
{
    double j0 = 0.0, j1 = 0.0, v0 = 0.0, v1 = 0.0;
    int off = 0;
    // JG joints at a time: their parameters are read after the previous group's terms (left to
    // itself the compiler hoisted all 84 LDS reads to the top: 168 registers live), and the group's
    // barrier chains interleave (one joint at a time, each v_rcp_f64 waited a wait state for its
    // reader: the trans forwarding hazard).  The sums add the joints in order either way.
#pragma unroll
    for (int j = 0; j < FR_NB; j += JG) {
        asm volatile("" : "+v"(off) : "v"(j < 6 ? j0 : j1));
        double lj[JG], lv[JG];
#pragma unroll
        for (int u = 0; u < JG; u++) {
            const double *P = Lj + off + u * JS;
            const double q = r[REC_QQD + 2 * (j + u)], vq = fabs(r[REC_QQD + 2 * (j + u) + 1]);
            lj[u] = left_barrier(P[0], P[1], P[2], q) + right_barrier(P[3], P[4], P[5], q);
            lv[u] = P[6] * (vq * vq);
        }
        off += JG * JS;
#pragma unroll
        for (int u = 0; u < JG; u++) {
            if (j + u < 6) { j0 += lj[u]; v0 += lv[u]; }
            else { j1 += lj[u]; v1 += lv[u]; }
        }
    }
    const double joint = j0 + j1, vel = v0 + v1;
    // the rest of the record (r holds the (q, qd) pairs only) is loaded through a pointer that
    // waits for the joint sums: the remaining terms start after them instead of interleaving with
    // them and holding their values live (two waves per SIMD instead of four)
    static_assert(REC_EE == 2 * FR_NB && REC_VL - REC_EE == 8, "record tail");
    // (the dependency rides on an index, not on the pointer: an opaque pointer loses its address
    // space, and its loads became flat_load, which wait for the LDS counter as well)
    double rest[REC_VL - REC_EE], yaw = r[REC_QQD + 4];
    int dep = 0;
    asm volatile("" : "+v"(dep), "+v"(yaw) : "v"(joint), "v"(vel));
    const double2 *tp = src + dep;
#pragma unroll
    for (int i = 0; i < (REC_VL - REC_EE) / 2; i++) {
        const double2 v = tp[REC_EE / 2 + i];
        rest[2 * i] = v.x;
        rest[2 * i + 1] = v.y;
    }
    double vl[3], jj[6];
    if constexpr (KC) {   // stored by the rows (REC_VL, REC_JJ)
        double kv[10];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const double2 v = tp[REC_VL / 2 + i];
            kv[2 * i] = v.x;
            kv[2 * i + 1] = v.y;
        }
#pragma unroll
        for (int i = 0; i < 3; i++) vl[i] = kv[i];
#pragma unroll
        for (int i = 0; i < 6; i++) jj[i] = kv[3 + i];
    } else {
        kin_sums(tp, vl, jj);   // from the stored record's motion subspaces
    }
    r = rest - REC_EE;   // r[REC_EE .. REC_VL) from here on
    double s, c;
    fsincos(yaw, &s, &c, sincos_constants());   // base yaw q_2
    const double *ee = r + REC_EE, *am = r + REC_AM;
    double wc = 0.0;
    {
        const double r22 = (1.0 - c) + c;
        const double fw0 = c, fw1 = s, fw2 = 0.0;
        const double off0 = (0.1 * c + (-s) * 0.0) + 0.0 * 0.15;
        const double off1 = (0.1 * s + c * 0.0) + 0.0 * 0.15;
        const double off2 = (0.0 * 0.1 + 0.0 * 0.0) + r22 * 0.15;
        const double rb2 = am[2] + off2;
        const double t0 = ee[0] - (am[0] + off0), t1 = ee[1] - (am[1] + off1), t2 = ee[2] - rb2;
        const double proj = ((t0 * fw0 + t1 * fw1) + t2 * fw2) / ((fw0 * fw0 + fw1 * fw1) + fw2 * fw2);
        wc += left_barrier(Cs.ws_infront, proj);
        wc += right_barrier(Cs.ws_reach, sqrt((t0 * t0 + t1 * t1) + t2 * t2));
        const double n1 = sqrt(t0 * t0 + t1 * t1);
        const double n2 = sqrt(fw0 * fw0 + fw1 * fw1);
        const double yaw = acos((t0 * fw0 + t1 * fw1) / n1 / n2);
        const double ay = fabs(yaw);
        const double yc = (Cs.yaw_c + Cs.yaw_l * fabs(ay)) + Cs.yaw_q * ay * ay;
        wc += isnan(yaw) ? 0.0 : yc;
        wc += left_barrier(Cs.ws_above, ee[2] - rb2);
    }
    double cost = 0.0;
    cost += Cs.en_joint ? joint : 0.0;
    cost += Cs.en_self ? Cs.self_collision : 0.0;
    cost += Cs.en_work ? wc : 0.0;
    if constexpr (EN) {   // energy_cost (:211-222)
        const double E = r[REC_E];
        cost += left_barrier(Cs.en_below, E) + right_barrier(Cs.en_above, E);
    }
    cost += Cs.en_vel ? vel : 0.0;
    cost += Cs.en_traj ? trajectory_term(Cs, sc, vl) : 0.0;
    cost += Cs.en_manip ? manipulability_term(Cs, jj) : 0.0;
    return cost;
}

// The seven terms of AssistedManipulation::get_cost at one step record (the whole record in r), as
// the reference's per-term accumulators see them (assisted_manipulation.cpp:74-319: m_joint_cost
// += ..., read back by get_joint_limit_cost() .. get_manipulability_cost(), .hpp:232-258): joint
// limits, self-collision, workspace, energy, velocity, trajectory, manipulability; a disabled
// term is 0 (get_cost skips it).  Same arithmetic as assisted_manipulation_cost; the optimal
// rollout's totals only (mppi_optimal_terms) and the standalone get_cost, so off the rollout
// kernels' path.  yaw: dynamics->get_state()[2] (workspace_cost, :160-168; in a rollout the
// record's q_2).
__device__ __forceinline__ void assisted_manipulation_terms(const DevCost &Cs, const StepConst &sc, const double *r, double yaw,
                                                            double *t)
{
    double j0 = 0.0, j1 = 0.0, v0 = 0.0, v1 = 0.0;
    for (int j = 0; j < FR_NB; j++) {
        const double q = r[REC_QQD + 2 * j], vq = fabs(r[REC_QQD + 2 * j + 1]);
        const double lj = left_barrier(Cs.lower[j], q) + right_barrier(Cs.upper[j], q);
        const double lv = Cs.vel_q[j] * (vq * vq);
        if (j < 6) { j0 += lj; v0 += lv; }
        else { j1 += lj; v1 += lv; }
    }
    double s, c;
    fsincos(yaw, &s, &c, sincos_constants());
    const double *ee = r + REC_EE, *am = r + REC_AM;
    double wc = 0.0;
    {
        const double r22 = (1.0 - c) + c;
        const double fw0 = c, fw1 = s, fw2 = 0.0;
        const double off0 = (0.1 * c + (-s) * 0.0) + 0.0 * 0.15;
        const double off1 = (0.1 * s + c * 0.0) + 0.0 * 0.15;
        const double off2 = (0.0 * 0.1 + 0.0 * 0.0) + r22 * 0.15;
        const double rb2 = am[2] + off2;
        const double t0 = ee[0] - (am[0] + off0), t1 = ee[1] - (am[1] + off1), t2 = ee[2] - rb2;
        const double proj = ((t0 * fw0 + t1 * fw1) + t2 * fw2) / ((fw0 * fw0 + fw1 * fw1) + fw2 * fw2);
        wc += left_barrier(Cs.ws_infront, proj);
        wc += right_barrier(Cs.ws_reach, sqrt((t0 * t0 + t1 * t1) + t2 * t2));
        const double n1 = sqrt(t0 * t0 + t1 * t1);
        const double n2 = sqrt(fw0 * fw0 + fw1 * fw1);
        const double ya = acos((t0 * fw0 + t1 * fw1) / n1 / n2);
        const double ay = fabs(ya);
        const double yc = (Cs.yaw_c + Cs.yaw_l * fabs(ay)) + Cs.yaw_q * ay * ay;
        wc += isnan(ya) ? 0.0 : yc;
        wc += left_barrier(Cs.ws_above, ee[2] - rb2);
    }
    const double E = r[REC_E];
    t[0] = Cs.en_joint ? j0 + j1 : 0.0;
    t[1] = Cs.en_self ? Cs.self_collision : 0.0;
    t[2] = Cs.en_work ? wc : 0.0;
    t[3] = Cs.en_energy ? left_barrier(Cs.en_below, E) + right_barrier(Cs.en_above, E) : 0.0;
    t[4] = Cs.en_vel ? v0 + v1 : 0.0;
    t[5] = Cs.en_traj ? trajectory_term(Cs, sc, r + REC_VL) : 0.0;
    t[6] = Cs.en_manip ? manipulability_term(Cs, r + REC_JJ) : 0.0;
}

// TrackPoint::get_cost: the joint terms sum joints 0..9 in order; reach_cost's robot point is the
// arm mount + R_z(yaw) (0.3, 0, 0.15) (track_point.cpp:162-186), yaw = dynamics->get_state()[2]
// (in a rollout the record's own q_2)
__device__ __forceinline__ double track_point_cost(const DevCost &Cs, const double *r, double yaw)
{
    const double *ee = r + REC_EE, *am = r + REC_AM;
    const double d0 = ee[0] - Cs.tp_point[0], d1 = ee[1] - Cs.tp_point[1], d2 = ee[2] - Cs.tp_point[2];
    const double distance = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    double cost = 100.0 * (distance * distance);   // point_cost: 100 pow(distance, 2)
    double joint = 0.0;
#pragma unroll
    for (int j = 0; j < 10; j++) {
        const double q = r[REC_QQD + 2 * j], lo = Cs.tp_lo[j], up = Cs.tp_up[j];
        const double below = (q < lo) ? 1000.0 + 100000.0 * ((lo - q) * (lo - q)) : 0.0;
        const double above = (q > up) ? 1000.0 + 100000.0 * ((q - up) * (q - up)) : 0.0;
        joint += below + above;
    }
    double s, c;
    fsincos(yaw, &s, &c, sincos_constants());
    const double r22 = (1.0 - c) + c;
    const double off0 = (0.3 * c + (-s) * 0.0) + 0.0 * 0.15;
    const double off1 = (0.3 * s + c * 0.0) + 0.0 * 0.15;
    const double off2 = (0.0 * 0.3 + 0.0 * 0.0) + r22 * 0.15;
    const double t0 = ee[0] - (am[0] + off0), t1 = ee[1] - (am[1] + off1), t2 = ee[2] - (am[2] + off2);
    const double reach = right_barrier(Cs.tp_reach, sqrt((t0 * t0 + t1 * t1) + t2 * t2));
    cost += Cs.tp_en_joint ? joint : 0.0;
    cost += Cs.tp_en_self ? Cs.tp_self : 0.0;
    cost += Cs.tp_en_reach ? reach : 0.0;
    return cost;
}

__device__ __forceinline__ double readlane_f64(double x, int l)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}

// gamma_k times the objective at step record r (AssistedManipulation: r holds the record's (q, qd)
// pairs, the rest is read from the stored record src; TrackPoint: r holds the record up to REC_VL)
template <int CK, bool EN, int JS = JT_STRIDE, bool KC = false, int JG = 1>
__device__ __forceinline__ double step_cost(const DevCost &Cs, const StepConst &sc, const double *r, const double *Lj,
                                           const double2 *src)
{
    if constexpr (CK == CK_TRACK_POINT) return sc.gamma_k * track_point_cost(Cs, r, r[REC_QQD + 4]);
    else return sc.gamma_k * assisted_manipulation_cost<EN, JS, KC, JG>(Cs, sc, r, Lj, src);
}

// gamma_k times the objective at the stored step record rk (FR_REC doubles, or FR_REC_C with KC;
// 16-byte aligned)
template <int CK, bool EN, int JS = JT_STRIDE, bool KC = false, int JG = 1>
__device__ __forceinline__ double record_step_cost(const DevCost &Cs, const StepConst &sc, const double *rk, const double *Lj)
{
    double r[FR_NREC];
    const double2 *src = reinterpret_cast<const double2 *>(rk);
    constexpr int NLOAD = CK == CK_TRACK_POINT ? REC_VL / 2 : FR_NB;   // AssistedManipulation: the (q, qd) pairs
#pragma unroll
    for (int i = 0; i < NLOAD; i++) {
        const double2 v = src[i];
        r[2 * i] = v.x;
        r[2 * i + 1] = v.y;
    }
    return step_cost<CK, EN, JS, KC, JG>(Cs, sc, r, Lj, src);
}

// J of one rollout from its H stored step records (rollout-major, FR_REC doubles each, FR_REC_C with
// KC) by one wave:
// lane k evaluates step k (64 steps a pass) and the wave sums the step costs in step order, as the
// reference accumulates J += cost (mppi.cpp:322-337); a NaN step makes the sum NaN (the reference's
// early stop), canonicalised to the quiet NaN it stores.  The same value on every lane.
template <int CK, bool EN, int JS = JT_STRIDE, bool KC = false>
__device__ __forceinline__ double rollout_cost(const DevCost &Cs, const StepConst *stp, const double *rec, int H, int lane,
                                               const double *Lj)
{
    constexpr int RS = KC ? FR_REC_C : FR_REC;
    double J = 0.0;
    for (int base = 0; base < H; base += 64) {
        const int n = (H - base < 64) ? H - base : 64;
        const int k = base + (lane < n ? lane : 0);
        const double c = record_step_cost<CK, EN, JS, KC>(Cs, stp[k], rec + (int64_t)k * RS, Lj);
        // J += c_i in step order; the lane reads eight at a time, ahead of their adds
        int i = 0;
        for (; i + 8 <= n; i += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = readlane_f64(c, i + u);
#pragma unroll
            for (int u = 0; u < 8; u++) J += v[u];
        }
        for (; i < n; i++) J += readlane_f64(c, i);
    }
    return isnan(J) ? (double)NAN : J;
}

// The costs' min / max / count (CostStats) gain one cost (NaN ones are not counted), in the slot
// of its rollout index
__device__ __forceinline__ void fold_cost_stats(CostStats *st, double J, int64_t r)
{
    if (!st || isnan(J)) return;
    const unsigned long long key = mppi_dev::cost_order_key(J);
    const int i = (int)(r & (CS_SLOTS - 1));
    atomicMin(&st->kmin[16 * i], key);
    atomicMax(&st->kmax[16 * i], key);
    atomicAdd(&st->count[32 * i], 1u);
}

}  // namespace mppi_cost
