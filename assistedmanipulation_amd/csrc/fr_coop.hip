// fr_coop.hip — cooperative FrankaRidgeback rollout kernel for gfx950.
//
// One rollout per DPP row (16 lanes), four rollouts per wave64.  The single-lane kernel in
// kernels.hip puts a whole rollout on one lane, which leaves 4098 rollouts on 65 waves (65 of
// the chip's 1024 SIMDs; one wave already saturates its SIMD's fp64 pipe).  Here the
// per-step work is spread over the row so 4098 rollouts fill ~1025 waves:
//
//   lane j (j < 12) owns joint / body j:  control component u_j, noise eps_j, q_j, qd_j,
//   sincos(q_j), its local transform, its world pose, motion subspace S_j and world inertia.
//
//   FK            inclusive prefix scan of SE3 products over the chain (row_shr 1,2,4,8),
//                 fingers 10/11 composed onto body 9 afterwards (row_newbcast:9)
//   kinematics    EE / arm-mount position (lanes 9 / 2), frame velocity J v and J_a J_a^T by
//                 16-lane DPP butterflies (quad_perm, row_half_mirror, row_mirror)
//   ABA backward  articulated inertia distributed by rows: lane r < 6 holds row r;
//                 world inertias / S_i staged in LDS by their owners; U, D, u by 8-lane sums
//   ABA forward   a (row-distributed), qdd_i by 8-lane sums, kept by lane i
//   cost          joint-limit / velocity terms per lane + one butterfly; workspace,
//                 trajectory and manipulability terms computed row-uniformly
//
// Semantics are those of fr_rollout_kernel (PinocchioDynamics::step + AssistedManipulation,
// one-step kinematic lag, NaN stop); only the association order of sums and products differs.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"

using namespace mppi_eng;
using mppi_dev::smax;
using mppi_dev::smin;

namespace {

constexpr int ROW = 16;
constexpr int ROWS_PER_WAVE = 4;
constexpr int COOP_NT = 64;                      // one wave per workgroup
// LDS per row (doubles): packed world inertias (21) and motion subspaces (6) of the 12 bodies,
// the backward pass's U (one per lane and body), 1/D and u (row-uniform, per body)
constexpr int L_I = 0;
constexpr int L_S = L_I + FR_NB * 21;
constexpr int L_U = L_S + FR_NB * 6;
constexpr int L_DU = L_U + FR_NB * ROW;
constexpr int LDS_ROW = L_DU + FR_NB * 2;
// per-block copy of the body table: per body R[9] p[3] mass c[3] Ic[6] frame_p[3]
constexpr int MB = 25;
constexpr int LDS_MODEL = FR_NB * MB;

// ---- DPP helpers (fp64 as two dwords) ------------------------------------------------------
// mov_dpp with bound_ctrl: lanes whose source lies outside the row read 0 (no `old` operand,
// so no zero-initialised destination register per move).
template <int CTRL>
__device__ __forceinline__ double dmov(double x)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
template <int N>
__device__ __forceinline__ double bcast(double x) { return dmov<0x150 + N>(x); }   // row_newbcast:N
template <int S>
__device__ __forceinline__ double shr(double x) { return dmov<0x110 + S>(x); }     // row_shr:S

// sum over the 16 lanes of a row; every lane gets the same bits (commutative pairwise adds)
__device__ __forceinline__ double rsum16(double x)
{
    x = x + dmov<0xB1>(x);    // quad_perm [1,0,3,2]
    x = x + dmov<0x4E>(x);    // quad_perm [2,3,0,1]
    x = x + dmov<0x141>(x);   // row_half_mirror
    x = x + dmov<0x140>(x);   // row_mirror
    return x;
}
// row_newbcast with a lane index that is a constant after unrolling
__device__ __forceinline__ double bcast_rt(double x, int n)
{
    switch (n) {
    case 0: return bcast<0>(x);
    case 1: return bcast<1>(x);
    case 2: return bcast<2>(x);
    case 3: return bcast<3>(x);
    case 4: return bcast<4>(x);
    case 5: return bcast<5>(x);
    case 6: return bcast<6>(x);
    case 7: return bcast<7>(x);
    case 8: return bcast<8>(x);
    case 9: return bcast<9>(x);
    case 10: return bcast<10>(x);
    default: return bcast<11>(x);
    }
}

__device__ __forceinline__ double right_barrier(double bound, double scale, double mx, double v)
{
    if (v >= bound) {
        const double d = v - bound;
        return mx + scale * (d * d);
    }
    return smin(scale / (bound - v), mx);
}
__device__ __forceinline__ double left_barrier(double bound, double scale, double mx, double v)
{
    if (v <= bound) {
        const double d = bound - v;
        return mx + scale * (d * d);
    }
    return smin(scale / (v - bound), mx);
}
__device__ __forceinline__ double left_barrier(const DevBarrier &b, double v) { return left_barrier(b.bound, b.scale, b.max, v); }
__device__ __forceinline__ double right_barrier(const DevBarrier &b, double v) { return right_barrier(b.bound, b.scale, b.max, v); }

// SE3 product (A.R B.R, A.p + A.R B.p)
__device__ __forceinline__ void compose(const double *Ra, const double *pa, double *R, double *p)
{
    double Rn[9], pn[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 3; c++) Rn[3 * r + c] = (Ra[3 * r] * R[c] + Ra[3 * r + 1] * R[3 + c]) + Ra[3 * r + 2] * R[6 + c];
        pn[r] = pa[r] + ((Ra[3 * r] * p[0] + Ra[3 * r + 1] * p[1]) + Ra[3 * r + 2] * p[2]);
    }
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = Rn[k];
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = pn[k];
}

template <int S>
__device__ __forceinline__ void scan_level(int j, double *R, double *p)
{
    double Rs[9], ps[3];
#pragma unroll
    for (int k = 0; k < 9; k++) Rs[k] = shr<S>(R[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) ps[k] = shr<S>(p[k]);
    if (j >= S && j < 10) compose(Rs, ps, R, p);
}

// Packed upper-triangle index of a symmetric 6x6.
__host__ __device__ constexpr int pidx(int r, int c)
{
    return (r <= c) ? (r * 6 - r * (r - 1) / 2 + (c - r)) : (c * 6 - c * (c - 1) / 2 + (r - c));
}

// World spatial inertia of the lane's body (packed 21), from its world pose; M = body table row.
__device__ __forceinline__ void world_inertia_to_lds(const double *M, const double *R, const double *p, double *dst)
{
    const double m = M[12];
    const double lc0 = M[13], lc1 = M[14], lc2 = M[15];
    double c[3];
#pragma unroll
    for (int r = 0; r < 3; r++) c[r] = ((R[3 * r] * lc0 + R[3 * r + 1] * lc1) + R[3 * r + 2] * lc2) + p[r];
    const double I00 = M[16], I01 = M[17], I11 = M[18], I02 = M[19], I12 = M[20], I22 = M[21];
    double RI[9];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        RI[3 * r + 0] = (R[3 * r] * I00 + R[3 * r + 1] * I01) + R[3 * r + 2] * I02;
        RI[3 * r + 1] = (R[3 * r] * I01 + R[3 * r + 1] * I11) + R[3 * r + 2] * I12;
        RI[3 * r + 2] = (R[3 * r] * I02 + R[3 * r + 1] * I12) + R[3 * r + 2] * I22;
    }
    const double mc0 = m * c[0], mc1 = m * c[1], mc2 = m * c[2];
    const double cc2 = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
    auto Iw = [&](int r, int s) { return (RI[3 * r] * R[3 * s] + RI[3 * r + 1] * R[3 * s + 1]) + RI[3 * r + 2] * R[3 * s + 2]; };
    // [[m E, -m[c]x], [m[c]x, Iw + m(|c|^2 E - c c^T)]], packed upper triangle
    dst[0] = m; dst[1] = 0.0; dst[2] = 0.0; dst[3] = 0.0; dst[4] = mc2; dst[5] = -mc1;
    dst[6] = m; dst[7] = 0.0; dst[8] = -mc2; dst[9] = 0.0; dst[10] = mc0;
    dst[11] = m; dst[12] = mc1; dst[13] = -mc0; dst[14] = 0.0;
    dst[15] = Iw(0, 0) + (m * cc2 - mc0 * c[0]);
    dst[16] = Iw(0, 1) - mc0 * c[1];
    dst[17] = Iw(0, 2) - mc0 * c[2];
    dst[18] = Iw(1, 1) + (m * cc2 - mc1 * c[1]);
    dst[19] = Iw(1, 2) - mc1 * c[2];
    dst[20] = Iw(2, 2) + (m * cc2 - mc2 * c[2]);
}

struct CoopKin {
    double ee[3], am[3], vl[3], jj[6];
};

// calculate(): FK by prefix scan, world inertias and S to LDS, the cost's kinematic cache.
__device__ __forceinline__ void coop_fk(int j, double q, double qd, const double *M, double *Lrow, CoopKin &kin)
{
    const int kind = j < FR_NB ? FR_KIND[j] : KIND_PX;
    const bool is_rz = kind == KIND_RZ;
    const int scol = (kind == KIND_PX) ? 0 : (is_rz ? 2 : 1);
    double R[9], p[3];
    if (is_rz) {
        double s, c;
        sincos(q, &s, &c);
#pragma unroll
        for (int r = 0; r < 3; r++) {
            R[3 * r + 0] = M[3 * r + 0] * c + M[3 * r + 1] * s;
            R[3 * r + 1] = M[3 * r + 0] * (-s) + M[3 * r + 1] * c;
            R[3 * r + 2] = M[3 * r + 2];
            p[r] = M[9 + r];
        }
    } else {
        const double qq = (kind == KIND_PNY) ? -q : q;
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int k = 0; k < 3; k++) R[3 * r + k] = M[3 * r + k];
            p[r] = M[9 + r] + M[3 * r + scol] * qq;
        }
    }
    scan_level<1>(j, R, p);
    scan_level<2>(j, R, p);
    scan_level<4>(j, R, p);
    scan_level<8>(j, R, p);
    {   // fingers hang off body 9
        double R9[9], p9[3];
#pragma unroll
        for (int k = 0; k < 9; k++) R9[k] = bcast<9>(R[k]);
#pragma unroll
        for (int k = 0; k < 3; k++) p9[k] = bcast<9>(p[k]);
        if (j == 10 || j == 11) compose(R9, p9, R, p);
    }
    double S[6];
    {
        const double c0 = R[scol], c1 = R[3 + scol], c2 = R[6 + scol];
        const double sg = (kind == KIND_PNY) ? -1.0 : 1.0;
        if (is_rz) {
            S[0] = p[1] * c2 - p[2] * c1;
            S[1] = p[2] * c0 - p[0] * c2;
            S[2] = p[0] * c1 - p[1] * c0;
            S[3] = c0;
            S[4] = c1;
            S[5] = c2;
        } else {
            S[0] = sg * c0;
            S[1] = sg * c1;
            S[2] = sg * c2;
            S[3] = 0.0;
            S[4] = 0.0;
            S[5] = 0.0;
        }
    }
    if (j < FR_NB) {
        world_inertia_to_lds(M, R, p, Lrow + L_I + j * 21);
#pragma unroll
        for (int k = 0; k < 6; k++) Lrow[L_S + j * 6 + k] = S[k];
    }
    double fpos[3];
#pragma unroll
    for (int r = 0; r < 3; r++) fpos[r] = p[r] + ((R[3 * r] * M[22] + R[3 * r + 1] * M[23]) + R[3 * r + 2] * M[24]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        kin.ee[k] = bcast<FR_EE_PARENT>(fpos[k]);
        kin.am[k] = bcast<FR_AM_PARENT>(fpos[k]);
    }
    const double wv = (j <= FR_EE_PARENT) ? qd : 0.0;
    const double wa = (j >= FR_ARM0 && j < FR_ARM1) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) kin.vl[k] = rsum16(S[k] * wv);
    const double w0 = wa * S[0], w1 = wa * S[1], w2 = wa * S[2];
    kin.jj[0] = rsum16(w0 * S[0]);
    kin.jj[1] = rsum16(w0 * S[1]);
    kin.jj[2] = rsum16(w0 * S[2]);
    kin.jj[3] = rsum16(w1 * S[1]);
    kin.jj[4] = rsum16(w1 * S[2]);
    kin.jj[5] = rsum16(w2 * S[2]);
}

// Articulated-body passes over the world inertias / S staged in LDS; returns qdd of the lane's
// joint.  The 6x6 articulated inertia is distributed by rows: lane j holds row j % 6 (lanes
// 6..15 duplicate rows 0..5, and row-uniform sums take lanes 0..5 only).
__device__ __forceinline__ double coop_aba(int j, double tau, double *Lrow)
{
    const int r = j % 6;
    const double rmask = j < 6 ? 1.0 : 0.0;
    int off[6];
#pragma unroll
    for (int c = 0; c < 6; c++) off[c] = pidx(r, c);
    double C[6], pA = 0.0;
#pragma unroll
    for (int k = 0; k < 6; k++) C[k] = 0.0;
#pragma unroll
    for (int i = FR_NB - 1; i >= 0; i--) {
        const double *Ii = Lrow + L_I + i * 21;
        const double *Si = Lrow + L_S + i * 6;
        double A[6], S[6];
#pragma unroll
        for (int k = 0; k < 6; k++) S[k] = Si[k];
        const double Sr = Si[r];
        if (i >= 10) {
#pragma unroll
            for (int k = 0; k < 6; k++) A[k] = Ii[off[k]];
        } else {
#pragma unroll
            for (int k = 0; k < 6; k++) A[k] = Ii[off[k]] + C[k];
        }
        const double pAr = (i >= 10) ? 0.0 : pA;
        double U = A[0] * S[0];
#pragma unroll
        for (int k = 1; k < 6; k++) U += A[k] * S[k];
        const double D = rsum16(rmask * (Sr * U));
        const double sp = rsum16(rmask * (Sr * pAr));
        const double Dinv = 1.0 / D;
        const double u = bcast_rt(tau, i) - sp;
        Lrow[L_U + i * ROW + j] = U;
        Lrow[L_DU + 2 * i] = Dinv;
        Lrow[L_DU + 2 * i + 1] = u;
        if (i > 0) {
            double Uall[6];
            Uall[0] = bcast<0>(U);
            Uall[1] = bcast<1>(U);
            Uall[2] = bcast<2>(U);
            Uall[3] = bcast<3>(U);
            Uall[4] = bcast<4>(U);
            Uall[5] = bcast<5>(U);
            const double Ud = U * Dinv;
            const double ud = u * Dinv;
            if (i == 10) {
#pragma unroll
                for (int k = 0; k < 6; k++) C[k] += A[k] - Ud * Uall[k];
                pA += pAr + U * ud;
            } else {
#pragma unroll
                for (int k = 0; k < 6; k++) C[k] = A[k] - Ud * Uall[k];
                pA = pAr + U * ud;
            }
        }
    }
    double acc = 0.0, a9 = 0.0, mine = 0.0;
#pragma unroll
    for (int i = 0; i < FR_NB; i++) {
        const double ap = (i == 11) ? a9 : acc;
        const double Sr = Lrow[L_S + i * 6 + r];
        const double ua = rsum16(rmask * (Lrow[L_U + i * ROW + j] * ap));
        const double dd = Lrow[L_DU + 2 * i] * (Lrow[L_DU + 2 * i + 1] - ua);
        acc = ap + Sr * dd;
        if (i == 9) a9 = acc;
        mine = (j == i) ? dd : mine;
    }
    return mine;
}

// t0 + k dt without FMA contraction (exact reference expression)
__device__ __forceinline__ double kdt(int k, double dt)
{
#pragma clang fp contract(off)
    return (double)k * dt;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(COOP_NT) void fr_coop_kernel(FrRolloutArgs a)
{
    __shared__ double lds[ROWS_PER_WAVE * LDS_ROW + LDS_MODEL];
    if (a.optimal && (a.status->all_nan || a.status->sg_error)) return;
    const int lane = threadIdx.x;
    const int j = lane & (ROW - 1);
    const int rowi = lane >> 4;
    double *Lrow = lds + rowi * LDS_ROW;
    double *Lmodel = lds + ROWS_PER_WAVE * LDS_ROW;
    {   // stage the body table: per body R p mass c Ic frame_p
        const DevModel &dm = *a.model;
        for (int t = lane; t < LDS_MODEL; t += COOP_NT) {
            const int b = t / MB, f = t % MB;
            const DevBody &db = dm.b[b];
            double v;
            if (f < 9) v = db.R[f];
            else if (f < 12) v = db.p[f - 9];
            else if (f == 12) v = db.mass;
            else if (f < 16) v = db.c[f - 13];
            else if (f < 22) v = db.Ic[f - 16];
            else v = (b == FR_EE_PARENT) ? dm.ee_p[f - 22] : ((b == FR_AM_PARENT) ? dm.am_p[f - 22] : 0.0);
            Lmodel[t] = v;
        }
        __syncthreads();
    }
    const int64_t lr = (int64_t)blockIdx.x * ROWS_PER_WAVE + rowi;   // local rollout of this row
    const bool live = lr < a.count;
    const int64_t g = a.optimal ? -1 : a.begin + lr;
    const int H = a.H;
    const int rank = (live && g >= 2) ? a.rank[g] : 0;
    const bool jl = j < FR_NB;      // lane owns a body / control component
    const int jb = jl ? j : 0;
    const double *M = Lmodel + jb * MB;
    const DevCost &Cs = *a.cost;
    const DevBarrier lo_b = Cs.lower[jb], up_b = Cs.upper[jb];
    const double vel_w = jl ? Cs.vel_q[jb] : 0.0;

    double q = live && jl ? a.x0[jb] : 0.0;
    double qd = live && jl ? a.x0[FR_NB + jb] : 0.0;
    CoopKin kin;
    coop_fk(j, q, qd, M, Lrow, kin);   // set_state -> calculate() at (q0, v0)
    double J = 0.0;
    bool alive = live;
    const double dt = a.dt;
    for (int k = 0; k < H; k++) {
        double eps = 0.0;
        if (!a.optimal && g != 0 && live && jl) {
            if (g == 1) {
                eps = -a.Uprev[k * FR_C + j];
            } else {
                const SampleParams &P = a.sp;
                int64_t draw = -1;
                if (rank < P.keep) {
                    if (P.shift_by > 0) {
                        if (k < P.shifted) eps = a.noise[((int64_t)(k + P.shift_by) * a.Rpad + lr) * FR_C + j];
                        else draw = (int64_t)rank * (H - P.shifted) + (k - P.shifted);
                    } else {
                        eps = a.noise[((int64_t)k * a.Rpad + lr) * FR_C + j];
                    }
                } else {
                    draw = P.keep_draws + (int64_t)(rank - P.keep) * H + k;
                }
                if (draw >= 0) {
                    if (P.injected) {
                        eps = a.inj[draw * FR_C + j];
                    } else {
                        const int blk = j >> 2;
                        mppi_dev::u32x4 ctr{(uint32_t)draw, (uint32_t)((uint64_t)draw >> 32), (uint32_t)P.update_index, (uint32_t)blk};
                        mppi_dev::u32x4 rr = mppi_dev::philox4x32_10(ctr, (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
                        float z0, z1;
                        if (j & 2) mppi_dev::box_muller(rr.z, rr.w, z0, z1);
                        else mppi_dev::box_muller(rr.x, rr.y, z0, z1);
                        const float z = (j & 1) ? z1 : z0;
                        if (P.tdiag) {
                            eps = a.T[j * FR_C + j] * (double)z;
                        } else {
                            eps = 0.0;
                            for (int c = 0; c < FR_C; c++) {
                                const double zc = __shfl((double)z, (lane & ~15) | c, 64);
                                eps += a.T[j * FR_C + c] * zc;
                            }
                        }
                    }
                }
            }
            a.noise[((int64_t)k * a.Rpad + lr) * FR_C + j] = eps;
        }
        if (!alive) continue;
        // cost at x_k with the kinematics cached by the previous calculate()
        const StepConst &sc = a.steps[k];
        double cost = 0.0;
        {
            const double lane_terms = (jl && Cs.en_joint) ? left_barrier(lo_b, q) + right_barrier(up_b, q) : 0.0;
            const double joint = rsum16(lane_terms);
            const double vq = fabs(qd);
            const double vel = rsum16(vel_w * (vq * vq));
            const double yawq = bcast<2>(q);
            if (Cs.en_joint) cost += joint;
            if (Cs.en_self) cost += Cs.self_collision;
            if (Cs.en_work) {
                double wc = 0.0;
                double s, c;
                sincos(yawq, &s, &c);
                const double r22 = (1.0 - c) + c;
                const double fw0 = c, fw1 = s, fw2 = 0.0;
                const double off0 = (0.1 * c + (-s) * 0.0) + 0.0 * 0.15;
                const double off1 = (0.1 * s + c * 0.0) + 0.0 * 0.15;
                const double off2 = (0.0 * 0.1 + 0.0 * 0.0) + r22 * 0.15;
                const double rb2 = kin.am[2] + off2;
                const double t0 = kin.ee[0] - (kin.am[0] + off0), t1 = kin.ee[1] - (kin.am[1] + off1), t2 = kin.ee[2] - rb2;
                const double proj = ((t0 * fw0 + t1 * fw1) + t2 * fw2) / ((fw0 * fw0 + fw1 * fw1) + fw2 * fw2);
                wc += left_barrier(Cs.ws_infront, proj);
                wc += right_barrier(Cs.ws_reach, sqrt((t0 * t0 + t1 * t1) + t2 * t2));
                const double n1 = sqrt(t0 * t0 + t1 * t1);
                const double n2 = sqrt(fw0 * fw0 + fw1 * fw1);
                const double yaw = acos((t0 * fw0 + t1 * fw1) / n1 / n2);
                if (!isnan(yaw)) {
                    const double ay = fabs(yaw);
                    wc += (Cs.yaw_c + Cs.yaw_l * fabs(ay)) + Cs.yaw_q * ay * ay;
                }
                wc += left_barrier(Cs.ws_above, kin.ee[2] - rb2);
                cost += wc;
            }
            if (Cs.en_vel) cost += vel;
            if (Cs.en_traj) {
                double tc = 0.0;
                if (sc.active) {
                    tc += sc.pos_cost;
                    double proj = ((kin.vl[0] * sc.target[0] + kin.vl[1] * sc.target[1]) + kin.vl[2] * sc.target[2]) / sc.tt;
                    const double p0 = proj * sc.target[0], p1 = proj * sc.target[1], p2 = proj * sc.target[2];
                    proj = copysign(1.0, proj) * sqrt((p0 * p0 + p1 * p1) + p2 * p2);
                    const double err = fabs(sc.vtarget - proj);
                    tc += (Cs.traj_vel_c + Cs.traj_vel_l * fabs(err)) + Cs.traj_vel_q * err * err;
                }
                cost += tc;
            }
            if (Cs.en_manip) {
                const double m00 = kin.jj[0], m01 = kin.jj[1], m02 = kin.jj[2], m11 = kin.jj[3], m12 = kin.jj[4], m22 = kin.jj[5];
                const double det = (m00 * (m11 * m22 - m12 * m12) - m01 * (m01 * m22 - m12 * m02)) + m02 * (m01 * m12 - m11 * m02);
                double vol = sqrt(det);
                if (isnan(vol)) vol = 1e-5;
                else vol = (vol < 1e-5) ? 1e-5 : ((1e5 < vol) ? 1e5 : vol);
                const double iv = 1.0 / vol;
                cost += (Cs.manip_c + Cs.manip_l * fabs(iv)) + Cs.manip_q * iv * iv;
            }
        }
        const double step_cost = sc.gamma_k * cost;
        if (!a.optimal && isnan(step_cost)) {
            J = NAN;
            alive = false;
            continue;
        }
        J += step_cost;
        if (k == H - 1) break;   // the final step's dynamics are never observed
        // PinocchioDynamics::step: base velocity overwrite, tau = arm controls, calculate, Euler
        const double u = (jl ? a.Ushift[k * FR_C + jb] : 0.0) + eps;
        {
            double s, c;
            sincos(bcast<2>(q), &s, &c);
            const double u0 = bcast<0>(u), u1 = bcast<1>(u);
            if (j == 0) qd = c * u0 + (-s) * u1;
            if (j == 1) qd = s * u0 + c * u1;
            if (j == 2) qd = u;
        }
        const double tau = (j >= 3 && j < 10) ? u : 0.0;
        coop_fk(j, q, qd, M, Lrow, kin);
        const double qdd = coop_aba(j, tau, Lrow);
        qd = qd + qdd * dt;
        q = q + qd * dt;
    }
    if (!live || j != 0) return;
    if (a.optimal) *a.cost_out = J;
    else a.cost_out[g] = J;
}

namespace mppi_eng {

hipError_t launch_fr_coop(const FrRolloutArgs &a, hipStream_t s)
{
    const unsigned nb = (unsigned)((a.count + ROWS_PER_WAVE - 1) / ROWS_PER_WAVE);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(fr_coop_kernel, dim3(nb), dim3(COOP_NT), 0, s, a);
    return hipGetLastError();
}

}  // namespace mppi_eng
