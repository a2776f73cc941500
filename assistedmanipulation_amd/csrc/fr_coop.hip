// fr_coop.hip — cooperative FrankaRidgeback rollout kernel for gfx950.
//
// One rollout per DPP row (16 lanes), four rollouts per wave64.  The single-lane kernel in
// kernels.hip puts a whole rollout on one lane, which leaves 4098 rollouts on 65 waves (65 of
// the chip's 1024 SIMDs).  Here the per-step work is spread over the row so 4098 rollouts fill
// ~1025 waves, one per SIMD:
//
//   lane j (j < 12) owns joint / body j:  control component u_j, eps_j, q_j, qd_j, sincos(q_j),
//   its local transform, world pose, motion subspace S_j and world inertia.  Lanes 12..15 run
//   the same instructions on a dummy body and are masked out of every sum and store.
//
//   FK            inclusive prefix scan of SE3 products over the lanes (row_shr 1,2,4,8) in
//                 delta form (R - I, p): the zeros row_shr shifts into lanes j < s are then the
//                 identity and the scan needs no masks.  Finger 11 hangs off body 9 like finger
//                 10; its placement is stored relative to finger 10's (DevModel::f11_*) and its
//                 local transform carries -q10, so its prefix world_10 * local_10^-1 * local_11
//                 is world_9 * local_11 without a second pass.
//   kinematics    EE / arm-mount positions (row_newbcast 9 / 2); frame velocity J v and J_a J_a^T
//                 as chains of v_fmac_f64_dpp row_newbcast (lane sums).
//   ABA           articulated inertia distributed by rows (lane r < 6 holds row r); world
//                 inertias / S / tau staged in LDS and read one level ahead; S.U, S.pA, the
//                 rank-1 update A - U U^T / D and the forward U.a are v_fmac_f64_dpp broadcasts.
//   records       every step's state and kinematics go to a per-rollout record array (kernels.hpp
//                 FR_NREC); fr_step_cost_kernel (fr_cost.hip) evaluates the objective on all of
//                 them, a lane per (rollout, step), and sums each rollout's costs in step order.
//                 The objective's terms are row-uniform, so inside this kernel all 16 lanes of a
//                 row would repeat them: moving them out cut the executed VALU work by 40 %.
//
// The step is written branch-free (selects, not branches) so the FK of step k and its record
// stores share basic blocks with the ABA chain and the scheduler can fill the chain's latency.
//
// Semantics are those of fr_rollout_kernel (PinocchioDynamics::step + AssistedManipulation,
// one-step kinematic lag, NaN stop); only the association order of sums and products differs.
// The rollout runs all H - 1 steps: a NaN step cost makes the rollout's sum NaN whatever follows.

#include <hip/hip_runtime.h>
#include <algorithm>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "fr_cost_terms.hpp"
#include "sample_device.hpp"
#include "fsincos.hpp"
#include <hip/hip_ext.h>

using namespace mppi_eng;
using mppi_dev::smax;
using mppi_dev::smin;

// PHASE_MARKS (analysis builds only, tools/phase_flops.py): a comment at each phase boundary of the
// step, so that the executed instructions can be attributed to phases - 0 the control and the base
// velocity, 1 FK (with the next step's sincos), 2 world inertias, 3 kinematics for the cost, 4 the
// composite inertias, 5 the mass-matrix columns, 6 the Gauss-Jordan solve, 7 integration and the
// record stores.  (A volatile asm ends the scheduler's region: the marked build is a little slower.)
// PMARK_D ties the marker to a value the next phase's inline-asm blocks consume or the previous
// one's produce: non-volatile asm statements are otherwise free to move across a plain marker.
// The body-table fields the step reads stay in registers across the horizon loop (REGTAB, round 6:
// 789 -> 766 instructions per step, no LDS re-read of the table in every step); -DNO_REGTAB for A/B
#ifndef NO_REGTAB
#define REGTAB 1
// (with it the compiler writes an F operand of column_dots right before the block: one wait state)
#define COLUMN_DOTS_PAD "s_nop 0\n\t"
#endif
#ifdef PHASE_MARKS
#define PMARK(n) asm volatile("; PHASE " #n)
#define PMARK_D(n, x) asm volatile("; PHASE " #n : "+v"(x))
#else
#define PMARK(n)
#define PMARK_D(n, x)
#endif

namespace {

constexpr int ROW = 16;
constexpr int ROWS_PER_WAVE = 4;
constexpr int CK_ASSISTED_MANIPULATION = 1, CK_TRACK_POINT = 3;   // mppi_cost_kind
constexpr int NSLOT = FR_NB + 1;   // + a dummy body slot that lanes 12..15 store into

// LDS per row (doubles).  Kinematic array (written by FK): packed world inertias (21) and motion
// subspaces (6) per body slot.  Scratch array (a separate object, so the compiler may move the
// backward pass's inertia reads over its scratch writes): U (per lane and body), 1/D and u
// (row-uniform, per body), qdd and tau per body.
// Row strides are 128 B modulo 256 B: ds_read_b64 serves lanes 0..31 (rows 0, 1) and 32..63 in
// one bank cycle each with bank (a/4) mod 64, so rows 0/1 (2/3) must sit half a bank sweep apart.
// Per-lane strides of the arrays that every lane of a row writes at once (mass-matrix rows, S
// slots) are 144 B and 80 B: their 16-byte stores then start at 36 j and 20 j (mod 64) dwords,
// sixteen disjoint four-bank groups per row.  With 128 B / 64 B strides the lanes of a row fell
// on two / four bank groups (8- / 4-way conflicts on the solve's transpose and the S stores).
constexpr int CSTR = 18;
constexpr int L_I = 0;
constexpr int L_COL = 0;                    // no tank: the mass-matrix block (16 x CSTR) over L_I
constexpr int L_TP = L_COL + 16 * CSTR;     // no tank: the solved right-hand side (12)
constexpr int L_S = 300;                    // 16-byte aligned; per slot S (6), qd, pad
constexpr int S_STR = 10;
// compact records without the tank (store_ks): per slot S linear x, y, z and qd, 48 B apart (the
// sixteen lanes' 16-byte stores start at 12 j (mod 64) dwords: disjoint bank groups); past the
// dummy lanes' 0 / 1 at L_TP + 12, 13 (with the tank store_ks reads coop_aba's L_S slots)
constexpr int L_KS = 304;
constexpr int KS_STR = 6;
constexpr int LDS_KIN = 432;                // >= L_S + NSLOT * S_STR, = 16 (mod 32) doubles
constexpr int L_F = 430;                    // energy tank: spatial force f of each body slot
constexpr int LDS_KIN_EN = 528;             // >= L_F + NSLOT * 6, = 16 (mod 32) doubles
constexpr int L_U = 0;
constexpr int L_DU = L_U + FR_NB * ROW;
constexpr int L_QDD = L_DU + FR_NB * 2;
constexpr int L_TAU = L_QDD + ROW;
constexpr int LDS_SCR = 272;                // >= L_TAU + ROW, = 16 (mod 32) doubles
static_assert(L_I + NSLOT * 21 <= L_S && L_S + NSLOT * S_STR <= LDS_KIN && L_TAU + ROW <= LDS_SCR, "LDS row layout");
// (L_TP + 12, 13: the dummy lanes' 0 / 1, over L_S, which only the tank's articulated-body pass uses)
static_assert(L_TP + 14 <= LDS_KIN && L_TP % 2 == 0, "LDS row layout (mass-matrix block)");
static_assert(L_S + NSLOT * S_STR <= L_F && L_F + NSLOT * 6 <= LDS_KIN_EN && L_F % 2 == 0, "LDS row layout (energy)");
static_assert(L_TP + 14 <= L_KS && L_KS % 2 == 0 && L_KS + NSLOT * KS_STR <= LDS_KIN, "LDS row layout (kinematic sums)");
static_assert(LDS_KIN % 32 == 16 && LDS_SCR % 32 == 16 && LDS_KIN_EN % 32 == 16, "row stride bank offset");

// Per-block body table (doubles per body): scan placement R p (body 11: relative to body 10),
// mass, com, inertia, frame offset (EE on body 9, arm mount on body 2), the placement's
// translation axis Ma = R a_t (prismatic joints; 0 for revolute), the joint axis a in the body
// frame, 1/0 for revolute / prismatic (and its complement), the joint-limit barriers and the
// velocity weight of the cost, and the lane masks of the kinematic sums.  Row 12 serves lanes
// 12..15: body 0's geometry with every mask and weight zero.
constexpr int T_R = 0, T_P = 9, T_M = 12, T_C = 13, T_IA = 16, T_IB = 19, T_F = 22, T_MA = 25, T_AX = 28, T_ROT = 31, T_NROT = 32;
constexpr int T_LO = 33, T_UP = 36, T_VW = 39, T_WV = 40, T_WA = 41, T_FIX = 42, T_MC = 43, T_IL = 44;
constexpr int MB = 45;   // odd: lanes reading their own body's entry hit distinct banks
constexpr int LDS_MODEL = (FR_NB + 1) * MB;
static_assert(LDS_MODEL <= FR_BODY_TABLE, "body table buffer");

// ---- DPP helpers (fp64 as two dwords) ------------------------------------------------------
// mov_dpp with bound_ctrl: lanes whose source lies outside the row read 0.
template <int CTRL>
__device__ __forceinline__ double dmov(double x)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
// row_newbcast:N as one v_mov_b64_dpp (gfx950's 64-bit DPP supports row_newbcast only)
template <int N>
__device__ __forceinline__ double bcast(double x) { return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + N, 0xF, 0xF, true); }
template <int S>
__device__ __forceinline__ double shr(double x) { return dmov<0x110 + S>(x); }     // row_shr:S

// acc + sum_{r<6} x[lane r] * y[r]: six v_fmac_f64_dpp row_newbcast:r (broadcast and multiply-add
// in one instruction; the compiler does not form 64-bit DPP FMAs).  The leading s_nop covers the
// VALU/EXEC-write -> DPP-read hazards.  Outputs are early-clobber ("+&v"): the blocks write the
// accumulator before their last read of x / y, so they must never share a register with an input
// (x and the accumulator are both the constant 0.0 at the finger levels of the ABA).
__device__ __forceinline__ double bfma6(double x, const double *y, double acc)
{
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "+&v"(acc)
        : "v"(x), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]));
    return acc;
}
// c[k] += x[lane k] * y for k < 6 (the rank-1 update of the articulated inertia rows)
__device__ __forceinline__ void bfma6_rank1(double x, double y, double *c)
{
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %6, %7 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %6, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %6, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %6, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %6, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "+&v"(c[0]), "+&v"(c[1]), "+&v"(c[2]), "+&v"(c[3]), "+&v"(c[4]), "+&v"(c[5])
        : "v"(x), "v"(y));
}
// sum over lanes [L0, L1) of x: v_fmac_f64_dpp row_newbcast:l with a unit multiplier (one asm
// block per range so the hazard nop stays in front of the chain)
template <int L0, int L1>
__device__ __forceinline__ double bsum(double x, double one);
template <>
__device__ __forceinline__ double bsum<0, 6>(double x, double one)
{
    const double ones[6] = {one, one, one, one, one, one};
    return bfma6(x, ones, 0.0);
}
template <>
__device__ __forceinline__ double bsum<0, 12>(double x, double one)
{
    double acc = 0.0;
    asm("s_nop 4\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf"
        : "+&v"(acc)
        : "v"(x), "v"(one));
    return acc;
}
// Interleaved chains.  A v_fmac_f64_dpp that accumulates into the result of the previous one waits
// ~14 cycles (no forwarding through a DPP instruction), while independent ones issue every ~5
// (tools/ubench.hip), so every block below round-robins several independent accumulators.
#define DPPF(acc, x, y, lane) "v_fmac_f64_dpp " acc ", " x ", " y " row_newbcast:" #lane " row_mask:0xf bank_mask:0xf\n\t"

// D = sum_{r<6} U[lane r] S[r] and sp = sum_{r<6} P[lane r] S[r]: two chains, interleaved (a
// four-chain split measured no faster: the extra zero-inits and adds cost what the shorter chains
// save).
__device__ __forceinline__ void bfma6_pair(double U, double P, const double *S, double &D, double &sp)
{
    double d0 = 0.0, p0 = 0.0;
    asm("s_nop 1\n\t"
        DPPF("%0", "%2", "%4", 0) DPPF("%1", "%3", "%4", 0) DPPF("%0", "%2", "%5", 1) DPPF("%1", "%3", "%5", 1)
        DPPF("%0", "%2", "%6", 2) DPPF("%1", "%3", "%6", 2) DPPF("%0", "%2", "%7", 3) DPPF("%1", "%3", "%7", 3)
        DPPF("%0", "%2", "%8", 4) DPPF("%1", "%3", "%8", 4) DPPF("%0", "%2", "%9", 5) DPPF("%1", "%3", "%9", 5)
        : "+&v"(d0), "+&v"(p0)
        : "v"(U), "v"(P), "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]));
    D = d0;
    sp = p0;
}
// sum over lanes 0..5 of x: two chains (lanes 0..2, 3..5)
__device__ __forceinline__ double bsum6_split(double x, double one)
{
    double a0 = 0.0, a1 = 0.0;
    asm("s_nop 1\n\t"
        DPPF("%0", "%2", "%3", 0) DPPF("%1", "%2", "%3", 3)
        DPPF("%0", "%2", "%3", 1) DPPF("%1", "%2", "%3", 4)
        DPPF("%0", "%2", "%3", 2) DPPF("%1", "%2", "%3", 5)
        : "+&v"(a0), "+&v"(a1)
        : "v"(x), "v"(one));
    return a0 + a1;
}
static_assert(FR_EE_PARENT == 9 && FR_ARM0 == 3 && FR_ARM1 == 10, "kinematic sum ranges");

// 1/d from v_rcp_f64 (2.5e8 ulp) by one quadratic correction r (1 + e + e^2), e = 1 - d r: three
// dependent FMAs instead of two Newton steps' four, and equal to the IEEE quotient on all 4M
// log-uniform samples of tools/rcp_probe.hip (d finite, normal)
__device__ __forceinline__ double frcp(double d)
{
    const double r = __builtin_amdgcn_rcp(d);
    const double e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, __builtin_fma(e, e, e), r);
}

// -x / d for the Gauss-Jordan pivots: v_rcp_f64 and one Newton correction applied to the product,
// t = -x r, e = 1 - d r, -x / d ~ t + t e (four ops, three deep; the rcp's 2.8e-8 relative error
// squares to ~1e-15).  frcp's exact reciprocal needs one more dependent FMA per pivot.
__device__ __forceinline__ double neg_quot(double x, double d)
{
    const double r = __builtin_amdgcn_rcp(d);
    const double t = -x * r;
    const double e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(t, e, t);
}

// b on the lanes whose mask m is all ones, a on the lanes where it is zero (m: a loop-invariant
// per-lane mask in a VGPR, made opaque where it is built).  One v_bfi_b32 per dword and no compare:
// C++ selects on the row index were compares per use, and LLVM turns a select whose operand is a
// load or a division into a branch - the step was ~40 basic blocks (exec-mask scaffolding that
// takes issue slots at one wave per SIMD, and scheduling regions the chains could not cross).
__device__ __forceinline__ double msel(int m, double a, double b)
{
    int lo, hi;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(m), "v"(__double2loint(b)), "v"(__double2loint(a)));
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(m), "v"(__double2hiint(b)), "v"(__double2hiint(a)));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int opaque_mask(bool c)
{
    int m = c ? -1 : 0;
    asm volatile("" : "+v"(m));
    return m;
}

// ---- BEGIN generated by tools/gen_gj.py: mass-matrix solve helpers ----
// m[i] = S_i . F for i = 0..9, S_i broadcast from lane i: rows 0 and 1 are F[0] and F[1] (the
// base's unit axes); rows 2..9 eight chains of six, round-robin, rows 3 and 7 on the lanes of
// the banks that hold their descendants only (bank_mask: the others keep 0); m[10] = 0 (body 10
// is nobody's ancestor)
__device__ __forceinline__ void column_dots(const double *S, const double *F, double *m)
{
    m[0] = F[0];
    m[1] = F[1];
#pragma unroll
    for (int i = 2; i < 11; i++) m[i] = 0.0;
    // no leading s_nop: S (the DPP sources) was formed long before (tools/dpp_hazard_check.py
    // checks every build's assembly; COLUMN_DOTS_PAD where a build puts an F write right before)
#ifndef COLUMN_DOTS_PAD
#define COLUMN_DOTS_PAD ""
#endif
    asm(COLUMN_DOTS_PAD
        "v_fmac_f64_dpp %0, %8, %14 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %14 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %8, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %8, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %8, %14 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %8, %14 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %8, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %9, %15 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %9, %15 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %9, %15 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %9, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %9, %15 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %9, %15 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %9, %15 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %9, %15 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %10, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %10, %16 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %10, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %10, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %10, %16 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %10, %16 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %10, %16 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %10, %16 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %11, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %11, %17 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %11, %17 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %11, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %11, %17 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %11, %17 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %11, %17 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %11, %17 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %12, %18 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %12, %18 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %12, %18 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %12, %18 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %12, %18 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %12, %18 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %12, %18 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %12, %18 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %13, %19 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %13, %19 row_newbcast:3 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %2, %13, %19 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %13, %19 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %13, %19 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %13, %19 row_newbcast:7 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %6, %13, %19 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %13, %19 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        : "+&v"(m[2]), "+&v"(m[3]), "+&v"(m[4]), "+&v"(m[5]), "+&v"(m[6]), "+&v"(m[7]), "+&v"(m[8]), "+&v"(m[9])
        : "v"(S[0]), "v"(S[1]), "v"(S[2]), "v"(S[3]), "v"(S[4]), "v"(S[5]), "v"(F[0]), "v"(F[1]), "v"(F[2]), "v"(F[3]), "v"(F[4]), "v"(F[5]));
}
// The twelve pivots of the Gauss-Jordan elimination, software-pipelined (pivot k's block
// updates row k + 1 first and interleaves pivot k + 1's reciprocal chain between its other
// FMAs), in one asm statement: nt is pivot 0's quotient, inv_next 1 / M[1][1]
__device__ __forceinline__ void gj_solve(double *Mc, double nt, double inv_next)
{
    double qa, qb, d, r, t, e;
    // s_nop 1: nt (a source of pivot 0's DPP FMAs) may be written right before the block
    asm("s_nop 1\n\t"
        /* pivot 0 */
        "v_fmac_f64_dpp %2, %2, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %12, -%1, %19\n\t"
        "v_fmac_f64_dpp %4, %4, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %18 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 1 */
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%2, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %9, %9, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %13, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 2 */
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%3, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %12, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 3 */
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%4, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %13, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 4 */
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%5, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %12, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 5 */
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%6, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %13, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 6 */
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%7, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %12, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 7 */
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%8, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %13, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 8 */
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%9, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %12, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 9 */
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%10, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %13, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 10 */
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %14, %11 row_newbcast:11 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %2, %2, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %15, %14\n\t"
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %16, -%11, %15\n\t"
        "v_fma_f64 %17, -%14, %15, 1.0\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %12, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 11 */
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        : "+v"(Mc[0]), "+v"(Mc[1]), "+v"(Mc[2]), "+v"(Mc[3]), "+v"(Mc[4]), "+v"(Mc[5]), "+v"(Mc[6]), "+v"(Mc[7]), "+v"(Mc[8]), "+v"(Mc[9]), "+v"(Mc[10]), "+v"(Mc[11]), "=&v"(qa), "=&v"(qb), "=&v"(d), "=&v"(r), "=&v"(t), "=&v"(e)
        : "v"(nt), "v"(inv_next));
}
#ifdef GJ_EXEC_NOP   // (A/B: wait states after each exec write, -DGJ_EXEC_NOP=n: s_nop n)
#define GJ_STR2(x) #x
#define GJ_STR(x) GJ_STR2(x)
#define GJ_EXEC_PAD "s_nop " GJ_STR(GJ_EXEC_NOP) "\n\t"
#else
#define GJ_EXEC_PAD ""
#endif
// Gauss-Jordan with one row per lane (tools/gen_gj.py solve_rows): Mc[0..11] row j of M, b
// tau_j; returns with b the solution on lanes 2..11 (rows normalised), b * m on lanes 0 and 1
// (scaled by 1 / m after).  f0 / f1: pivot 0 / 1's factors (-M_j0 / m0, -M_j1 / m1; 0 on lane
// 0 / 1).  Exec is saved, narrowed for the factors of each pivot and restored inside.
__device__ __forceinline__ void gj_rows(double *Mc, double &b, double f0, double f1)
{
    double fa, fb, d, r0, e, q;
    uint64_t sx, mk;
    const uint64_t base = 0x0001000100010001ull;   // lane 0 of each 16-lane row
    // (no leading s_nop: tools/dpp_hazard_check.py checks every build that Mc / f0 / f1, DPP
    // operands, were not written in the two instructions before the block)
    asm(""
        "s_mov_b64 %19, exec\n\t"
        "s_lshl_b64 %20, %23, 2\n\t"
        /* pivot 0 */
        "v_fmac_f64_dpp %2, %2, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %21 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 1 */
        "v_fmac_f64_dpp %2, %2, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %5, %5, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %6, %6, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %7, %7, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %8, %8, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %13, -%2, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %13, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 3\n\t"
        "v_fmac_f64_dpp %11, %11, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %22 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 2 */
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %14, -%3, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %14, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 4\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 3 */
        "v_fmac_f64_dpp %4, %4, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %7, %7, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %8, %8, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %9, %9, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_fmac_f64_dpp %10, %10, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f64 %13, -%4, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %13, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 5\n\t"
        "v_fmac_f64_dpp %11, %11, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 4 */
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %14, -%5, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %14, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 6\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 5 */
        "v_fmac_f64_dpp %6, %6, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %9, %9, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %10, %10, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %11, %11, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %13, -%6, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %13, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 7\n\t"
        "v_fmac_f64_dpp %12, %12, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        /* pivot 6 */
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fmac_f64_dpp %12, %12, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %14, -%7, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %14, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 8\n\t"
        /* pivot 7 */
        "v_fmac_f64_dpp %8, %8, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %9, %9, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %11, %11, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "v_fmac_f64_dpp %12, %12, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %13, -%8, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %13, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 9\n\t"
        /* pivot 8 */
        "v_fmac_f64_dpp %9, %9, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %10, %10, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f64_dpp %12, %12, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "s_nop 0\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %14, -%9, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %14, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 10\n\t"
        /* pivot 9 */
        "v_fmac_f64_dpp %10, %10, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %11, %11, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b64_dpp %15, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "s_nop 0\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %13, -%10, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %13, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        "s_lshl_b64 %20, %23, 11\n\t"
        /* pivot 10 */
        "v_fmac_f64_dpp %11, %11, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %12, %12, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_mov_b64_dpp %15, %11 row_newbcast:11 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_rcp_f64 %16, %15\n\t"
        "s_nop 0\n\t"
        "v_fma_f64 %17, -%15, %16, 1.0\n\t"
        "v_fma_f64 %18, %16, %17, %16\n\t"
        "v_mul_f64 %14, -%11, %18\n\t"
        "s_and_b64 exec, %19, %20\n\t" GJ_EXEC_PAD
        "v_add_f64 %14, %18, -1.0\n\t"
        "s_mov_b64 exec, %19\n\t" GJ_EXEC_PAD
        /* pivot 11 */
        "s_nop 0\n\t"
        "v_fmac_f64_dpp %12, %12, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        : "+v"(Mc[0]), "+v"(Mc[1]), "+v"(Mc[2]), "+v"(Mc[3]), "+v"(Mc[4]), "+v"(Mc[5]), "+v"(Mc[6]), "+v"(Mc[7]), "+v"(Mc[8]), "+v"(Mc[9]), "+v"(Mc[10]), "+v"(Mc[11]), "+v"(b), "=&v"(fa), "=&v"(fb), "=&v"(d), "=&v"(r0), "=&v"(e), "=&v"(q), "=&s"(sx), "=&s"(mk)
        : "v"(f0), "v"(f1), "s"(base)
        : "scc");
}
// ---- END generated by tools/gen_gj.py ----

// A rotation's third column from its first two, r2 = r0 x r1 (R row-major).
__device__ __forceinline__ void rot_col2(double *R)
{
    R[2] = R[3] * R[7] - R[6] * R[4];
    R[5] = R[6] * R[1] - R[0] * R[7];
    R[8] = R[0] * R[4] - R[3] * R[1];
}

// One level of the prefix scan in delta form (D = R - I, p): the partner's pose (Da, pa) arrives by
// row_shr S - its rotation's first two columns and translation, 9 doubles (18 moves) - and
//   (I + Da)(I + D) = I + Da + Ra D,   pa + Ra p,   Ra = I + Da,
// with Ra's third column the cross product of its first two.  Each entry is one FMA chain that
// starts from the partner's term (3 operations), and only columns 0 and 1 are formed; the lane's own
// third column is never read before the end of the scan.  Lanes the shift leaves without a partner
// receive zeros: Ra = I, pa = 0, the identity.  (r04: Da + D + Da D with the partner's third column
// rebuilt in delta form, 61 operations a level; r05: 53.)
template <int S>
__device__ __forceinline__ void scan_level2(double *D, double *p)
{
    double Ra[9], Da[6], pa[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        Da[2 * r] = shr<S>(D[3 * r]);
        Da[2 * r + 1] = shr<S>(D[3 * r + 1]);
        pa[r] = shr<S>(p[r]);
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
        Ra[3 * r] = Da[2 * r];
        Ra[3 * r + 1] = Da[2 * r + 1];
    }
    Ra[0] += 1.0;
    Ra[4] += 1.0;
    rot_col2(Ra);
    double Dn[6], pn[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 2; c++)
            Dn[2 * r + c] = __builtin_fma(Ra[3 * r], D[c], __builtin_fma(Ra[3 * r + 1], D[3 + c],
                                          __builtin_fma(Ra[3 * r + 2], D[6 + c], Da[2 * r + c])));
        pn[r] = __builtin_fma(Ra[3 * r], p[0], __builtin_fma(Ra[3 * r + 1], p[1], __builtin_fma(Ra[3 * r + 2], p[2], pa[r])));
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
        D[3 * r] = Dn[2 * r];
        D[3 * r + 1] = Dn[2 * r + 1];
        p[r] = pn[r];
    }
}

// The scan's last level (row_shr 8) for this robot: what lanes 8..11 compose with is the world pose of
// bodies 0..3 (the planar base and panda_joint1), which is a rotation about z and a translation
// (check_topology rejects any model where it is not).  So only (cos - 1, sin) of that rotation and
// its translation travel - 5 doubles (10 moves) instead of 9 - and the product is
// Dw + (I + Dw) D with Dw = [[dc, -s, 0], [s, dc, 0], [0, 0, 0]]: 14 operations.
// Lanes 0..7 receive zeros, the identity.  (The partner's R11, -R01 are taken as its R00, R10: equal
// for a z rotation up to the last bit of the scan's rounding.)
__device__ __forceinline__ void scan_level_planar8(double *D, double *p)
{
    const double dc = shr<8>(D[0]), sn = shr<8>(D[3]);
    const double pw0 = shr<8>(p[0]), pw1 = shr<8>(p[1]), pw2 = shr<8>(p[2]);
    const double cw = dc + 1.0;
    const double d00 = D[0], d01 = D[1], d10 = D[3], d11 = D[4];
    D[0] = __builtin_fma(cw, d00, __builtin_fma(-sn, d10, dc));
    D[1] = __builtin_fma(cw, d01, __builtin_fma(-sn, d11, -sn));
    D[3] = __builtin_fma(sn, d00, __builtin_fma(cw, d10, sn));
    D[4] = __builtin_fma(sn, d01, __builtin_fma(cw, d11, dc));
    const double p0 = p[0], p1 = p[1];
    p[0] = __builtin_fma(cw, p0, __builtin_fma(-sn, p1, pw0));
    p[1] = __builtin_fma(sn, p0, __builtin_fma(cw, p1, pw1));
    p[2] = p[2] + pw2;
}

// Packed upper-triangle index of a symmetric 6x6.
__host__ __device__ constexpr int pidx(int r, int c)
{
    return (r <= c) ? (r * 6 - r * (r - 1) / 2 + (c - r)) : (c * 6 - c * (c - 1) / 2 + (r - c));
}

// World spatial inertia of the lane's body, from its world pose (M = body table row): world com c,
// rotational inertia about the com Iw, and Ib = Iw + m (|c|^2 E - c c^T), the angular block about
// the origin (packed xx xy xz yy yz zz); with h = m c the 6x6 is [[m E, -[h]x], [[h]x, Ib]].
// The body inertia about the com is held in rank-2 form, I = l E + a a^T + b b^T (l its least
// eigenvalue, a and b the other two eigenvectors scaled by the square roots of their excess over
// l: inertia_rank2, in the body table), so R I R^T = l E + (R a)(R a)^T + (R b)(R b)^T: two
// rotated vectors and two FMAs an entry (40 operations for Ib against 55 for R I R^T).  The energy
// variant's articulated-body pass reads Ib from LDS, packed upper triangle (21), and its RNEA
// forces take Iw (IW); without it the parallel-axis term seeds Ib's chains and Iw is not formed.
template <bool IW>
__device__ __forceinline__ void world_inertia(const double *M, const double *R, const double *p, double *c, double *Iw,
                                              double *Ib)
{
    const double m = M[T_M];
    const double lc0 = M[T_C], lc1 = M[T_C + 1], lc2 = M[T_C + 2];
    double ra[3], rb[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        c[r] = __builtin_fma(R[3 * r + 2], lc2, __builtin_fma(R[3 * r + 1], lc1, __builtin_fma(R[3 * r], lc0, p[r])));
        ra[r] = __builtin_fma(R[3 * r + 2], M[T_IA + 2], __builtin_fma(R[3 * r + 1], M[T_IA + 1], R[3 * r] * M[T_IA]));
        rb[r] = __builtin_fma(R[3 * r + 2], M[T_IB + 2], __builtin_fma(R[3 * r + 1], M[T_IB + 1], R[3 * r] * M[T_IB]));
    }
    const double l = M[T_IL];
    const double mc0 = m * c[0], mc1 = m * c[1], mc2 = m * c[2];
    const double cc2 = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
    // entry (u, v) of (R a)(R a)^T + (R b)(R b)^T, from x
    auto ab = [&](int u, int v, double x) { return __builtin_fma(ra[u], ra[v], __builtin_fma(rb[u], rb[v], x)); };
    if constexpr (IW) {
        Iw[0] = ab(0, 0, l);
        Iw[1] = ab(0, 1, 0.0);
        Iw[2] = ab(0, 2, 0.0);
        Iw[3] = ab(1, 1, l);
        Iw[4] = ab(1, 2, 0.0);
        Iw[5] = ab(2, 2, l);
        const double mcc = m * cc2;
        Ib[0] = Iw[0] + (mcc - mc0 * c[0]);
        Ib[1] = Iw[1] - mc0 * c[1];
        Ib[2] = Iw[2] - mc0 * c[2];
        Ib[3] = Iw[3] + (mcc - mc1 * c[1]);
        Ib[4] = Iw[4] - mc1 * c[2];
        Ib[5] = Iw[5] + (mcc - mc2 * c[2]);
    } else {
        const double mcl = __builtin_fma(m, cc2, l);   // m |c|^2 + l, the diagonal's common part
        Ib[0] = ab(0, 0, __builtin_fma(-mc0, c[0], mcl));
        Ib[1] = ab(0, 1, -mc0 * c[1]);
        Ib[2] = ab(0, 2, -mc0 * c[2]);
        Ib[3] = ab(1, 1, __builtin_fma(-mc1, c[1], mcl));
        Ib[4] = ab(1, 2, -mc1 * c[2]);
        Ib[5] = ab(2, 2, __builtin_fma(-mc2, c[2], mcl));
    }
}
__device__ __forceinline__ void inertia_to_lds(double m, const double *c, const double *Ib, double *dst)
{
    const double mc0 = m * c[0], mc1 = m * c[1], mc2 = m * c[2];
    // [[m E, -m[c]x], [m[c]x, Ib]], packed upper triangle
    dst[0] = m; dst[1] = 0.0; dst[2] = 0.0; dst[3] = 0.0; dst[4] = mc2; dst[5] = -mc1;
    dst[6] = m; dst[7] = 0.0; dst[8] = -mc2; dst[9] = 0.0; dst[10] = mc0;
    dst[11] = m; dst[12] = mc1; dst[13] = -mc0; dst[14] = 0.0;
    dst[15] = Ib[0]; dst[16] = Ib[1]; dst[17] = Ib[2]; dst[18] = Ib[3]; dst[19] = Ib[4]; dst[20] = Ib[5];
}

// Inclusive prefix sum over the row's lanes of a 6-vector (Hillis-Steele, row_shr 1, 2, 4, 8).
__device__ __forceinline__ void prefix6(double *x)
{
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] += shr<1>(x[k]);
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] += shr<2>(x[k]);
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] += shr<4>(x[k]);
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] += shr<8>(x[k]);
}
__device__ __forceinline__ void cross3(const double *a, const double *b, double *o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
// Spatial inertia (mass m, world com c, rotational inertia Iw about the com, packed xx xy xz yy
// yz zz) times a motion [v; w] at the world origin: [m (v + w x c); Iw w + c x m (v + w x c)].
__device__ __forceinline__ void inertia_mul(double m, const double *c, const double *Iw, const double *x, double *h)
{
    double wc[3], vc[3], ch[3];
    cross3(x + 3, c, wc);
#pragma unroll
    for (int k = 0; k < 3; k++) { vc[k] = x[k] + wc[k]; h[k] = m * vc[k]; }
    cross3(c, h, ch);
    h[3] = ((Iw[0] * x[3] + Iw[1] * x[4]) + Iw[2] * x[5]) + ch[0];
    h[4] = ((Iw[1] * x[3] + Iw[3] * x[4]) + Iw[4] * x[5]) + ch[1];
    h[5] = ((Iw[2] * x[3] + Iw[4] * x[4]) + Iw[5] * x[5]) + ch[2];
}

// What the cost of the next step needs from a calculate() (row-uniform): EE and arm-mount
// positions, written to the step record.  (The EE frame velocity J v and J_a J_a^T are formed by
// the objective from the record's motion subspaces: store_kin.)
struct CoopKin {
    double fp[3];   // the lane's frame position (store_record: EE on lane FR_EE_PARENT, arm mount on FR_AM_PARENT)
    double pw;   // energy tank: f . V of the lane's body (NLE power at the pre-step velocity)
};

// The mass-matrix solve's inputs from a calculate(): the lane's world motion subspace and its body's
// world spatial inertia as (m, h = m c, Ib) (zero on lanes 12..15).
struct CoopBody {
    double S[6], m, h[3], Ib[6];
};

// Lane-constant data of the row's body j (the doubles live in the body table).
struct LaneConst {
    int slot;       // LDS body slot (dummy for lanes 12..15)
    bool is_rz;
    double rz, nrz;   // is_rz as 1.0 / 0.0 and its complement: the joint rotation's (cos, sin) by one FMA
                      // and one multiply instead of four v_cndmask_b32
    // opaque lane masks (0 / -1) for msel, built once before the horizon loop
    int m_j12, m_j13, m_j14, m_j15;   // j == n
    // lane coefficients (1.0 / 0.0, opaque): base_velocity's, and tau_u's (3 <= j < 10: the arm
    // joints it drives)
    double bA, bB, bnA, bC, bkeep, taud;
    int ka, kb;     // store_ks (compact records): kinematic sum min(j, 8)'s x and y offsets in a body's LDS slot
    int m_vsum;     // store_ks: the sum is a J v row (bodies 0..9), else a J_a J_a^T entry (bodies 3..9)
    int rec_off;    // store_record: the lane's (q, qd) slot, 2 j, or REC_E for the dummy lanes
    int fp_off;     // store_record: REC_EE / REC_AM on lanes FR_EE_PARENT / FR_AM_PARENT, else REC_FP_SINK
    double ancd[10];   // the same as 1.0 / 0.0 (rows 3 and 7 unused: bank masks): column_dots' entries are finite, so a product masks
    double cmask[9];   // composite_scan: 1.0 when body j is the parent of step s's child (edges 11-9, 10-9, 9-8, .., 3-2)
    double mc;      // the mass of body j's subtree (composite inertia's mass, a constant)
    double inv_m0, inv_m1;   // 1 / composite mass of bodies 0 and 1: the base pivots (uniform)
    double f0, f1;  // gj_rows: pivot 0 / 1's factor per unit of M_j0 / M_j1 (-1 / m; 0 on lane 0 / 1)
    double qs;      // gj_rows: the solution's scale (1 / m on lanes 0 and 1, else 1)
};

// calculate(): FK by prefix scan, world inertias and S to LDS, the next cost's kinematic terms.
template <int CK, bool EN>
__device__ __forceinline__ void coop_fk(const LaneConst &L, double q, double sq, double cq, double qd, const double *M,
                                        double *Lk, CoopKin &kin, CoopBody &bd, const double *grav)
{
    PMARK(1);
    const double cz = __builtin_fma(L.rz, cq, L.nrz);   // cq on revolute lanes, 1 elsewhere
    const double sz = L.rz * sq;                         // sq on revolute lanes, 0 elsewhere
    const double qprev = shr<1>(q);
    // delta form D = R - I (columns 0 and 1; the scan never reads the third): the diagonal's -1 is
    // the seed of its FMA chain
    double D[9], p[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double m0 = M[T_R + 3 * r], m1 = M[T_R + 3 * r + 1];
        D[3 * r + 0] = r == 0 ? __builtin_fma(m0, cz, __builtin_fma(m1, sz, -1.0)) : m0 * cz + m1 * sz;
        D[3 * r + 1] = r == 1 ? __builtin_fma(m1, cz, __builtin_fma(-m0, sz, -1.0)) : m0 * (-sz) + m1 * cz;
        D[3 * r + 2] = 0.0;
        p[r] = M[T_P + r] + M[T_MA + r] * q;
    }
    p[1] = p[1] + M[T_FIX] * qprev;
    scan_level2<1>(D, p);
    scan_level2<2>(D, p);
    scan_level2<4>(D, p);
    scan_level_planar8(D, p);
    double R[9];
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = D[k];
    R[0] += 1.0;
    R[4] += 1.0;
    rot_col2(R);
    // motion subspace: revolute (p x w, w), prismatic (w, 0), w = R a
    double w[3], S[6];
#pragma unroll
    for (int r = 0; r < 3; r++) w[r] = (R[3 * r] * M[T_AX] + R[3 * r + 1] * M[T_AX + 1]) + R[3 * r + 2] * M[T_AX + 2];
    const double rotf = M[T_ROT], nrotf = M[T_NROT];
    S[3] = w[0] * rotf;
    S[4] = w[1] * rotf;
    S[5] = w[2] * rotf;
    // p x (w rotf) + w nrotf: the same bits as (p x w) rotf + w nrotf on both kinds of lane
    S[0] = __builtin_fma(p[1], S[5], __builtin_fma(-p[2], S[4], w[0] * nrotf));
    S[1] = __builtin_fma(p[2], S[3], __builtin_fma(-p[0], S[5], w[1] * nrotf));
    S[2] = __builtin_fma(p[0], S[4], __builtin_fma(-p[1], S[3], w[2] * nrotf));
    double com[3], Iw[6], Ib[6];
    PMARK(2);
    world_inertia<EN>(M, R, p, com, Iw, Ib);
    if constexpr (EN) inertia_to_lds(M[T_M], com, Ib, Lk + L_I + L.slot * 21);   // coop_aba's input
    {   // lanes 12..15: the table's dummy body has zero mass and inertia, so h = Ib = 0 there
        bd.m = M[T_M];
#pragma unroll
        for (int k = 0; k < 3; k++) bd.h[k] = M[T_M] * com[k];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            bd.Ib[k] = Ib[k];
            bd.S[k] = S[k];
        }
    }
    kin.pw = 0.0;
    if constexpr (EN) {
        // coop_aba's motion subspaces (the mass-matrix solve takes them from registers)
#pragma unroll
        for (int k = 0; k < 6; k++) Lk[L_S + L.slot * S_STR + k] = S[k];
        Lk[L_S + L.slot * S_STR + 6] = qd;
        // The energy tank's power needs tau = tau_u + nonLinearEffects(q, v) (pinocchio_dynamics.cpp:
        // 156, 248-251).  With W_j = sum_{i <= j} S_i v_new,i, NLE . v_new = sum_j f_j . W_j where
        // f_j = I_j A_j + V_j x* I_j V_j is body j's RNEA force (world frame, at the origin):
        //   V_j = sum_{i <= j} S_i qd_i,   A_j = -g + sum_{i <= j} V_i x S_i qd_i   (prefix sums)
        // and W_j = V_j + dt sum_{i <= j} S_i qdd_i: the f . V part is summed here, the qdd part in
        // the ABA's forward pass (coop_aba).  Finger 11's prefix drops finger 10's term.
        double xs[6], V[6], cA[6];
#pragma unroll
        for (int k = 0; k < 6; k++) xs[k] = S[k] * qd;
#pragma unroll
        for (int k = 0; k < 6; k++) V[k] = xs[k] + M[T_FIX] * shr<1>(xs[k]);
        prefix6(V);
        double t0[3], t1[3];
        cross3(V + 3, xs, t0);
        cross3(V, xs + 3, t1);
        cross3(V + 3, xs + 3, cA + 3);
#pragma unroll
        for (int k = 0; k < 3; k++) cA[k] = t0[k] + t1[k];
        double A[6];
#pragma unroll
        for (int k = 0; k < 6; k++) A[k] = cA[k] + M[T_FIX] * shr<1>(cA[k]);
        prefix6(A);
#pragma unroll
        for (int k = 0; k < 3; k++) A[k] -= grav[k];
        const double m = M[T_M];
        double hA[6], hV[6], f[6];
        inertia_mul(m, com, Iw, A, hA);
        inertia_mul(m, com, Iw, V, hV);
        // V x* h = [w x h_lin; w x h_ang + v x h_lin]
        double g0[3], g1[3], g2[3];
        cross3(V + 3, hV, g0);
        cross3(V + 3, hV + 3, g1);
        cross3(V, hV, g2);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            f[k] = hA[k] + g0[k];
            f[3 + k] = hA[3 + k] + (g1[k] + g2[k]);
        }
#pragma unroll
        for (int k = 0; k < 6; k++) Lk[L_F + L.slot * 6 + k] = f[k];
        kin.pw = ((f[0] * V[0] + f[1] * V[1]) + f[2] * V[2]) + ((f[3] * V[3] + f[4] * V[4]) + f[5] * V[5]);
    }
    // the frame at offset T_F of the lane's body: the EE on lane FR_EE_PARENT, the arm mount on lane
    // FR_AM_PARENT (zero offset elsewhere), for store_record
    PMARK(3);
#pragma unroll
    for (int r = 0; r < 3; r++)
        kin.fp[r] = __builtin_fma(R[3 * r + 2], M[T_F + 2], __builtin_fma(R[3 * r + 1], M[T_F + 1], __builtin_fma(R[3 * r], M[T_F], p[r])));
}

// The record's motion subspaces for the objective's J v and J_a J_a^T (kernels.hpp REC_S01 /
// REC_S2Q, fr_cost_terms.hpp kin_sums): the lane's S linear part and the qd its calculate() used,
// two 16-byte stores per lane (lanes 12..15 and the fingers into slots nobody reads).  Until r05 the
// row formed the nine sums itself after the FK - S and qd through LDS, ten LDS-read FMAs and the
// base's selects per lane, ~45 instructions on the dynamics chain of every step; the objective's
// waves now run the same FMA chains beside the loops, in the issue slots one wave leaves idle.
template <int CK>
__device__ __forceinline__ void store_kin(double *rp, int j, const CoopBody &bd, double qd)
{
    if constexpr (CK == CK_TRACK_POINT) return;   // TrackPoint reads the EE / arm-mount positions only
    *reinterpret_cast<double2 *>(rp + REC_S01 + 2 * j) = double2{bd.S[0], bd.S[1]};
    *reinterpret_cast<double2 *>(rp + REC_S2Q + 2 * j) = double2{bd.S[2], qd};
}

// The compact record's kinematics (fr_coop_kernel, FR_REC_C): the row forms the nine sums itself -
// the EE frame velocity J v over bodies 0..9 and J_a J_a^T over the arm (3..9) - lane m = min(j, 8)
// sum m from the S / qd slots the row writes to LDS, in the order and with the FMAs of the objective's
// kin_sums (fr_cost_terms.hpp: i = 0..9, acc = fma(x_i, y_i, acc), y_i = 0 for the base's J_a J_a^T),
// so the costs keep their bits.  About 40 instructions on the chain of every step (r04's form): where
// a wave evaluates its own rows' objective after its loop there are no objective waves beside the
// loops to absorb them, and the record, written and read back, is half the 768-B one's bytes.
// EN: the tank kernel's layout (coop_aba's L_S slots, qd at 6); STAGED: coop_fk<CK, true> wrote them
// (every step of the tank kernel but the set_state calculate() before its loop)
template <int CK, bool EN, bool STAGED = EN>
__device__ __forceinline__ void store_ks(double *rp, int j, const LaneConst &L, const CoopBody &bd, double qd, double *Lk)
{
    if constexpr (CK == CK_TRACK_POINT) return;   // TrackPoint reads the EE / arm-mount positions only
    constexpr int B = EN ? L_S : L_KS, ST = EN ? S_STR : KS_STR;
    if constexpr (!EN) {
        *reinterpret_cast<double2 *>(Lk + L_KS + L.slot * KS_STR) = double2{bd.S[0], bd.S[1]};
        *reinterpret_cast<double2 *>(Lk + L_KS + L.slot * KS_STR + 2) = double2{bd.S[2], qd};
    } else if constexpr (!STAGED) {
        *reinterpret_cast<double2 *>(Lk + L_S + L.slot * S_STR) = double2{bd.S[0], bd.S[1]};
        Lk[L_S + L.slot * S_STR + 2] = bd.S[2];
        Lk[L_S + L.slot * S_STR + 6] = qd;
    }
    const double *xs = Lk + B + L.ka, *ys = Lk + B + L.kb;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i <= FR_EE_PARENT; i++) {
        double y = ys[i * ST];
        if (i < FR_ARM0) y = msel(L.m_vsum, 0.0, y);
        acc = __builtin_fma(xs[i * ST], y, acc);
    }
    rp[REC_VL + (j < 9 ? j : 8)] = acc;   // lanes 9..15 repeat lane 8: same address, same value
}

// Articulated-body passes over the world inertias / S staged in LDS (energy-tank rollouts, whose
// power needs the forward pass's spatial accelerations; the others use coop_solve); returns qdd of
// the lane's joint.  Backward pass: the 6x6 articulated inertia is distributed by rows (lane r < 6
// holds row r; lanes 6..15 mirror row 5, unused); U = A S per row, D = S.U and S.pA as DPP
// broadcast-FMA chains, and the rank-1 update A_parent = (A + I_parent) - U U^T / D with the
// parent's own inertia added before the update.  Forward pass per level: qdd_i = (u_i - U_i . a_p)
// / D_i, a_i = a_p + S_i qdd_i.
template <bool EN>
__device__ __forceinline__ double coop_aba(int j, const double *Lk, double *Lw, double &pe)
{
    const int r = j < 6 ? j : 5;   // lanes 0..5 hold rows 0..5; the others mirror row 5, unused
    int off[6];
#pragma unroll
    for (int c = 0; c < 6; c++) off[c] = pidx(r, c);
    // operands of the next level are loaded one level ahead (LDS latency off the chain)
    double An[6], Sn[6], taun;
    auto fetch = [&](int i) {
        const double *Ii = Lk + L_I + i * 21;
        const double *Si = Lk + L_S + i * S_STR;
#pragma unroll
        for (int k = 0; k < 6; k++) An[k] = Ii[off[k]];
#pragma unroll
        for (int k = 0; k < 6; k++) Sn[k] = Si[k];
        taun = Lw[L_TAU + i];
    };
    fetch(FR_NB - 1);
    double A[6], C[6], pA = 0.0;
#pragma unroll
    for (int i = FR_NB - 1; i >= 0; i--) {
        double S[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            if (i >= 10) A[k] = An[k];      // finger leaves
            else if (i == 9) A[k] = C[k];   // C: the fingers' parts plus body 9's own inertia
            S[k] = Sn[k];
        }
        const double tau = taun;
        if (i > 0) fetch(i - 1);
        const double pAr = (i >= 10) ? 0.0 : pA;
        const double U = ((A[0] * S[0] + A[1] * S[1]) + (A[2] * S[2] + A[3] * S[3])) + (A[4] * S[4] + A[5] * S[5]);
        // D = S.U and S.pA: rows 0..5 broadcast from lanes 0..5, every lane holds S
        double D, sp;
        bfma6_pair(U, pAr, S, D, sp);
        const double Dinv = frcp(D);
        const double u = tau - sp;
        Lw[L_U + i * ROW + j] = U;
        Lw[L_DU + 2 * i] = Dinv;
        Lw[L_DU + 2 * i + 1] = u;
        if (i > 0) {
            const double Ud = U * Dinv;
            const double ud = u * Dinv;
            // parent's articulated inertia, row r: (A + I_parent)[k] - (U_r / D) U_k
            if (i == 11) {   // first finger: parent 9 is reached through finger 10's level
#pragma unroll
                for (int k = 0; k < 6; k++) C[k] = A[k];
                pA = pAr + U * ud;
                bfma6_rank1(U, -Ud, C);
            } else if (i == 10) {   // An now holds body 9 (fetched above)
#pragma unroll
                for (int k = 0; k < 6; k++) C[k] = (C[k] + A[k]) + An[k];
                pA += pAr + U * ud;
                bfma6_rank1(U, -Ud, C);
            } else {
#pragma unroll
                for (int k = 0; k < 6; k++) A[k] = A[k] + An[k];
                pA = pAr + U * ud;
                bfma6_rank1(U, -Ud, A);
            }
        }
    }
    pe = 0.0;
    {
        double acc = 0.0, a9 = 0.0;
        double Srf = Lk[L_S + r], Uf = Lw[L_U + j], Dvf = Lw[L_DU], uf = Lw[L_DU + 1];
        double Ff = EN ? Lk[L_F + r] : 0.0;
#pragma unroll
        for (int i = 0; i < FR_NB; i++) {
            const double Sr = Srf, Ui = Uf, Dv = Dvf, ui = uf, Fr = Ff;
            if (i + 1 < FR_NB) {
                Srf = Lk[L_S + (i + 1) * S_STR + r];
                Uf = Lw[L_U + (i + 1) * ROW + j];
                Dvf = Lw[L_DU + 2 * (i + 1)];
                uf = Lw[L_DU + 2 * (i + 1) + 1];
                if constexpr (EN) Ff = Lk[L_F + (i + 1) * 6 + r];
            }
            const double ap = (i == 11) ? a9 : acc;
            const double ua = bsum6_split(Ui * ap, 1.0);
            const double dd = Dv * (ui - ua);
            acc = ap + Sr * dd;
            if (i == 9) a9 = acc;
            if constexpr (EN) pe += Fr * acc;   // row r of f_i . sum_{k <= i} S_k qdd_k
            Lw[L_QDD + i] = dd;
        }
        const double qdd = Lw[L_QDD + (j < FR_NB ? j : 0)];
        return j < FR_NB ? qdd : 0.0;
    }
}


// Composite inertia (h, Ib) of the lane's subtree, summed in place from the leaves up: each edge
// (child i -> parent p) of the tree is one step v_c += v_c[lane i] m, m = 1.0 on lane p only, in an
// order that finishes every child before it is read (fingers 11 and 10 into body 9, then 9 into 8,
// ..., 3 into 2).  Nine steps of nine v_fmac_f64_dpp, the components interleaved, so each read of a
// lane's value comes nine instructions after its write (two wait states are the DPP rule; the
// dependency waits out the rest).  Bodies 0 and 1 (the base's prismatic joints) need no composite:
// their columns of M are the constant composite mass on the diagonal (S_0, S_1 unit translations),
// whatever h and Ib hold.  (r04: the whole subtree of each lane by broadcasts from lanes 2..11, ninety
// FMAs plus nine zeroed accumulators; r05: 81 FMAs into the lanes' own values, nothing to zero.)
__device__ __forceinline__ void composite_scan(double *v, const double *m)
{
    // (no leading s_nop: tools/dpp_hazard_check.py checks every build that the lanes' own (h, Ib),
    // the DPP sources, were not written in the two instructions before the block)
    asm(""
        "v_fmac_f64_dpp %0, %0, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %0, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %1, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %2, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %3, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %4, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %5, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %6, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %7, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %8, %8, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8])
        : "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]), "v"(m[6]), "v"(m[7]), "v"(m[8]));
}

// PinocchioDynamics::step's base velocity overwrite (pinocchio_dynamics.cpp): lane 0 takes
// vx = c u0 - s u1, lane 1 vy = s u0 + c u1 (c, s: the base yaw's, lane 2; u0, u1: lanes 0, 1),
// lane 2 u itself, the other lanes keep qd.  As lane coefficients: P = A c + B s, Q = B c - A s,
// qd' = (C u + u0 P) + (keep qd + u1 Q), six broadcast FMAs in place of four broadcasts, four
// products and three two-way selects.  The order keeps two instructions between a VGPR's write and
// a DPP instruction's read of it (one s_nop where nothing else fits).
__device__ __forceinline__ double base_velocity(const LaneConst &L, double u, double sq, double cq, double qd)
{
    double P = 0.0, Q = 0.0, X, Y;
    asm(
#ifdef REGTAB
        "s_nop 1\n\t"
#endif
        "v_fmac_f64_dpp %0, %5, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"    // P = c A
        "v_fmac_f64_dpp %1, %5, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"    // Q = c B
        "v_mul_f64 %2, %11, %6\n\t"                                                  // X = C u
        "v_mul_f64 %3, %12, %7\n\t"                                                  // Y = keep qd
        "v_fmac_f64_dpp %0, %4, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"    // P += s B
        "v_fmac_f64_dpp %1, %4, %10 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"   // Q += s (-A)
        "s_nop 0\n\t"
        "v_fmac_f64_dpp %2, %6, %0 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"    // X += u0 P
        "v_fmac_f64_dpp %3, %6, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf"          // Y += u1 Q
        : "+&v"(P), "+&v"(Q), "=&v"(X), "=&v"(Y)
        : "v"(sq), "v"(cq), "v"(u), "v"(qd), "v"(L.bA), "v"(L.bB), "v"(L.bnA), "v"(L.bC), "v"(L.bkeep));
    return X + Y;
}

// Mass-matrix solve for the rollouts without the energy tank: qdd = M(q)^-1 tau_u, M by the
// composite-rigid-body algorithm in world coordinates and eliminated by Gauss-Jordan, one column
// per lane.  Equal to the zero-bias articulated-body pass in exact arithmetic; its serial chain is
// twelve scalar pivots (the pivot d_k is already on lane k) instead of twelve 6x6 levels whose
// D = S^T A S needs a six-deep cross-lane chain each.
//   composite inertia   Ic_j = sum over the subtree of j, as (m, h, Ib): a suffix sum over lanes
//                       0..11 (row_shl 1, 2, 4, 8); finger 10's subtree is itself.
//   column j            M_ij = S_i . Ic_j S_j for the ancestors i of j (S_i broadcast from lane i),
//                       M_jj on the diagonal; the entries below the diagonal by symmetry through
//                       LDS.  Lane 12 holds the right-hand side tau.
//   Gauss-Jordan        twelve pivots, each one broadcast of the pivot, a reciprocal and eleven
//                       broadcast FMAs per lane; then qdd_j = tau'_j / M'_jj.
__device__ __forceinline__ double coop_solve(int j, const LaneConst &L, const CoopBody &bd, double tau_l, double *Lk)
{
    // (h, Ib) summed over the subtree; the subtree's mass is a per-lane constant of the body table (T_MC)
    double v[9] = {bd.h[0], bd.h[1], bd.h[2], bd.Ib[0], bd.Ib[1], bd.Ib[2], bd.Ib[3], bd.Ib[4], bd.Ib[5]};
#pragma unroll
    for (int i = 0; i < 9; i++) PMARK_D(4, v[i]);
    composite_scan(v, L.cmask);
#pragma unroll
    for (int i = 0; i < 9; i++) PMARK_D(5, v[i]);
    // F = Ic S: [m v - h x w; h x v + Ib w], S = (v; w)
    const double *S = bd.S;
    const double m = L.mc, h0 = v[0], h1 = v[1], h2 = v[2];
    const double I00 = v[3], I01 = v[4], I02 = v[5], I11 = v[6], I12 = v[7], I22 = v[8];
    double F[6];
    F[0] = m * S[0] - (h1 * S[5] - h2 * S[4]);
    F[1] = m * S[1] - (h2 * S[3] - h0 * S[5]);
    F[2] = m * S[2] - (h0 * S[4] - h1 * S[3]);
    F[3] = (h1 * S[2] - h2 * S[1]) + ((I00 * S[3] + I01 * S[4]) + I02 * S[5]);
    F[4] = (h2 * S[0] - h0 * S[2]) + ((I01 * S[3] + I11 * S[4]) + I12 * S[5]);
    F[5] = (h0 * S[1] - h1 * S[0]) + ((I02 * S[3] + I12 * S[4]) + I22 * S[5]);
    double Mc[12];
    column_dots(S, F, Mc);
    const double diag = ((S[0] * F[0] + S[1] * F[1]) + (S[2] * F[2] + S[3] * F[3])) + (S[4] * F[4] + S[5] * F[5]);
    // strictly-upper part of column j: M_ij for the ancestors i of j (finger 11 hangs off body 9,
    // not finger 10), zero elsewhere; lanes 12..15 have F = 0 and so a zero column.  Rows 3 and 7
    // come masked by column_dots' bank masks and row 10 as zero (nobody's ancestor).
#pragma unroll
    for (int i = 0; i < 10; i++)
        if (i != 3 && i != 7) Mc[i] *= L.ancd[i];
    Mc[11] = 0.0;
    // row j of the block: that column, then tau_j and zeros in slots 12..15, then the diagonal over
    // slot j (LDS stores of a wave land in order).  Entry (i, j) of the block is then column i's
    // row-j entry: M_ji = M_ij below the diagonal, the diagonal, and zero above it - so column j is
    // its strictly-upper part plus a read of block column j, with no select; lane 12 reads the
    // right-hand side tau, lanes 13..15 zeros.
    double *Row = Lk + L_COL + j * CSTR;
#pragma unroll
    for (int i = 0; i < 12; i += 2) *reinterpret_cast<double2 *>(Row + i) = double2{Mc[i], Mc[i + 1]};
#ifdef GJ_COLS
    Row[12] = tau_l;   // (slots 13..15: zeros for good, coop_rows' entry)
#endif
    Row[j] = diag;
#pragma unroll
    for (int i = 0; i < 12; i++) Mc[i] += Lk[L_COL + i * CSTR + j];
#pragma unroll
    for (int i = 0; i < 12; i++) PMARK_D(6, Mc[i]);
#ifndef GJ_COLS
    // one row per lane (M symmetric: the column is the row), tau_j the lane's own right-hand side;
    // lanes 12..15 read zeros (slots 12..15 of every block row) and have tau 0, so their b stays 0
    double b = tau_l;
    gj_rows(Mc, b, Mc[0] * L.f0, Mc[1] * L.f1);
    return b * L.qs;   // rows 2..11 normalised; rows 0 and 1 times 1 / m
#else
    double nt = -Mc[0] * L.inv_m0;   // each pivot's block returns the next pivot's quotient
    gj_solve(Mc, nt, L.inv_m1);
    // The matrix is now diagonal (every row scaled alike): qdd_j = tau'_j / M'_jj.  Lane 12 leaves
    // tau' at L_TP and every other lane its column in its own block row (read above, dead now), so
    // lane j reads M'_jj back at slot j of that row: no per-lane register select, no branch.
    double *dst = (j == 12) ? Lk + L_TP : Row;
#pragma unroll
    for (int i = 0; i < 12; i += 2) *reinterpret_cast<double2 *>(dst + i) = double2{Mc[i], Mc[i + 1]};
    // Lanes 12..15 read 0 / 1 (L_TP + 12, 13, coop_rows' entry): qdd = 0, q = qd = 0 for good
    const double tp = Lk[j < FR_NB ? L_TP + j : L_TP + 12];
    const double dj = Lk[j < FR_NB ? L_COL + j * CSTR + j : L_TP + 13];
    return tp * frcp(dj);
#endif
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// The per-body table (geometry, inertia, axes, cost weights, lane masks), built once per handle
// (launch_fr_body_table, at create: the model and cost are constants of the handle).  Built in the
// rollout kernels themselves, its chain of dependent, divergent loads of the model held every
// workgroup for ~7 us before its first step (PRO_TRACE); a copy of the table is one load.
// A symmetric 3x3 inertia (packed xx xy yy xz yz zz, DevBody::Ic) as l E + a a^T + b b^T: cyclic
// Jacobi rotations to its eigenvalues / vectors, l the least eigenvalue, a and b the other two
// eigenvectors times sqrt(lambda - l) (inertias are positive semi-definite, so l >= 0 and the two
// excesses are >= 0; rounding is clamped).
__device__ void inertia_rank2(const double *Ic, double *a, double *b, double *l)
{
    double A[3][3] = {{Ic[0], Ic[1], Ic[3]}, {Ic[1], Ic[2], Ic[4]}, {Ic[3], Ic[4], Ic[5]}};
    double V[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    for (int sweep = 0; sweep < 32; sweep++) {
        const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
        if (off == 0.0) break;
        for (int pq = 0; pq < 3; pq++) {
            const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
            if (A[p][q] == 0.0) continue;
            const double th = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
            const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; k++) {   // A <- A J (columns p, q)
                const double akp = A[k][p], akq = A[k][q];
                A[k][p] = c * akp - s * akq;
                A[k][q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; k++) {   // A <- J^T A (rows p, q)
                const double apk = A[p][k], aqk = A[q][k];
                A[p][k] = c * apk - s * aqk;
                A[q][k] = s * apk + c * aqk;
            }
            A[p][q] = A[q][p] = 0.0;
            for (int k = 0; k < 3; k++) {   // V <- V J
                const double vkp = V[k][p], vkq = V[k][q];
                V[k][p] = c * vkp - s * vkq;
                V[k][q] = s * vkp + c * vkq;
            }
        }
    }
    int lo = 0;
    for (int i = 1; i < 3; i++)
        if (A[i][i] < A[lo][lo]) lo = i;
    const int i1 = lo == 0 ? 1 : 0, i2 = lo == 2 ? 1 : 2;
    *l = A[lo][lo];
    const double sa = sqrt(fmax(A[i1][i1] - *l, 0.0)), sb = sqrt(fmax(A[i2][i2] - *l, 0.0));
    for (int k = 0; k < 3; k++) {
        a[k] = sa * V[k][i1];
        b[k] = sb * V[k][i2];
    }
}

__global__ void fr_body_table_kernel(const DevModel *model, const DevCost *cost, double *table)
{
    const DevModel &dm = *model;
    const DevCost &dc = *cost;
    for (int t = threadIdx.x; t < LDS_MODEL; t += blockDim.x) {
        const int row = t / MB, f = t % MB;
        const bool dummy = row == FR_NB;
        const int b = dummy ? 0 : row;
        const DevBody &db = dm.b[b];
        const int kind = FR_KIND[b];
        const double *Rs = (b == 11) ? dm.f11_R : db.R;
        const double *ps = (b == 11) ? dm.f11_p : db.p;
        // translation axis a_t (prismatic; 0 for revolute) and joint axis a, body frame
        const double ax0 = (kind == KIND_PX) ? 1.0 : 0.0;
        const double ax1 = (kind == KIND_PY) ? 1.0 : ((kind == KIND_PNY) ? -1.0 : 0.0);
        const double ax2 = (kind == KIND_RZ) ? 1.0 : 0.0;
        const double live = dummy ? 0.0 : 1.0;
        double v;
        if (f < T_P) v = Rs[f];
        else if (f < T_M) v = ps[f - T_P];
        else if (f == T_M) v = live * db.mass;   // the dummy body (lanes 12..15) is massless:
        else if (f < T_IA) v = live * db.c[f - T_C];   // its world inertia, F and M column vanish
        else if (f < T_F || f == T_IL) {   // the rotational inertia in rank-2 form (inertia_rank2)
            double ia[3], ib[3], il;
            inertia_rank2(db.Ic, ia, ib, &il);
            v = live * (f == T_IL ? il : (f < T_IB ? ia[f - T_IA] : ib[f - T_IB]));
        }
        else if (f < T_MA) v = (b == FR_EE_PARENT) ? dm.ee_p[f - T_F] : ((b == FR_AM_PARENT) ? dm.am_p[f - T_F] : 0.0);
        else if (f < T_AX) {
            const int r = f - T_MA;
            v = Rs[3 * r] * ax0 + Rs[3 * r + 1] * ax1;   // a_t = a for prismatic joints (PX, PY, PNY)
        } else if (f == T_AX) v = ax0;
        else if (f == T_AX + 1) v = ax1;
        else if (f == T_AX + 2) v = ax2;
        else if (f == T_ROT) v = (kind == KIND_RZ) ? live : 0.0;
        else if (f == T_NROT) v = (kind == KIND_RZ) ? 0.0 : live;
        else if (f < T_UP) v = live * ((f == T_LO) ? dc.lower[b].bound : (f == T_LO + 1) ? dc.lower[b].scale : dc.lower[b].max);
        else if (f < T_VW) v = live * ((f == T_UP) ? dc.upper[b].bound : (f == T_UP + 1) ? dc.upper[b].scale : dc.upper[b].max);
        else if (f == T_VW) v = live * dc.vel_q[b];
        else if (f == T_WV) v = (!dummy && b <= FR_EE_PARENT) ? 1.0 : 0.0;
        else if (f == T_WA) v = (!dummy && b >= FR_ARM0 && b < FR_ARM1) ? 1.0 : 0.0;
        else if (f == T_FIX) v = (!dummy && b == 11) ? -1.0 : 0.0;
        else if (f == T_MC) {   // the composite mass of the body's subtree (a constant: no scan)
            v = 0.0;
            for (int i = b; i < FR_NB && !dummy; i++)
                if (b <= FR_EE_PARENT || i == b) v += dm.b[i].mass;
        } else v = 0.0;
        table[t] = v;
    }
}

// Stage the body table in LDS.
__device__ __forceinline__ void stage_body_table(const FrRolloutArgs &a, double *Lmodel, int nt)
{
    for (int t = threadIdx.x; t < LDS_MODEL; t += nt) Lmodel[t] = a.table[t];
}

// Step record store (layout: kernels.hpp FR_REC), the whole row active (no branch splits the
// step's basic block): lanes 0..11 write (q_j, qd_j) and lanes 12..15 the EE / arm-mount
// positions and the tank energy (one 16-byte store), then lane j writes kinematic sum min(j, 8)
// (the motion subspaces for the objective's sums: store_kin, after the FK).
template <bool EN>
__device__ __forceinline__ void store_record(double *rp, int j, const LaneConst &L, double q, double qd, const CoopKin &kin,
                                             double E)
{
    if constexpr (!EN) {
        // Without the tank E = 0, and the dummy lanes 12..15 hold q = qd = 0: they store their pair
        // over slots 30..31 (E, pad), which hold zeros either way, so no select builds their part of
        // the record.  The EE / arm-mount / E slots are row-uniform values that every lane of the row
        // stores alike (the same bytes to the same addresses): four stores instead of sixteen
        // v_bfi_b32.
        // two 8-byte stores (relaxed wavefront-scope atomics: plain stores the vectorizer leaves
        // apart) - a 16-byte one needs (q, qd) in adjacent registers, two v_mov_b32 per step
        __hip_atomic_store(rp + L.rec_off, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_store(rp + L.rec_off + 1, qd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        // the EE and arm-mount positions from the lanes that own them; the other lanes' frame
        // positions go to slots nobody reads (REC_FP_SINK)
        double *f = rp + L.fp_off;
        f[0] = kin.fp[0];
        f[1] = kin.fp[1];
        f[2] = kin.fp[2];
        return;   // (slots 30, 31 - E, pad: the dummy lanes' zero pair)
    }
    double ee[3], am[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        ee[k] = bcast<FR_EE_PARENT>(kin.fp[k]);
        am[k] = bcast<FR_AM_PARENT>(kin.fp[k]);
    }
    double a0 = msel(L.m_j12, q, ee[0]), a1 = msel(L.m_j12, qd, ee[1]);
    a0 = msel(L.m_j13, a0, ee[2]);
    a1 = msel(L.m_j13, a1, am[0]);
    a0 = msel(L.m_j14, a0, am[1]);
    a1 = msel(L.m_j14, a1, am[2]);
    a0 = msel(L.m_j15, a0, E);
    a1 = msel(L.m_j15, a1, 0.0);
    *reinterpret_cast<double2 *>(rp + 2 * j) = double2{a0, a1};
}
// slots 88..90: S2Q's entries of the dummy lanes 12..15, written by store_kin and read by nobody
// (the compact record's: REC_SINK_C)
constexpr int REC_FP_SINK = REC_S2Q + 2 * 12;
static_assert(REC_VL + 9 <= REC_SINK_C && REC_SINK_C + 3 <= FR_REC_C && FR_REC_C % 16 == 0 && FR_NREC <= FR_REC_C,
              "compact record layout");
static_assert(REC_EE == 24 && REC_AM == 27 && REC_E == 30 && REC_S01 == 32 && REC_S2Q == 64 && FR_REC == 96, "record layout");
static_assert(REC_FP_SINK + 3 <= FR_REC, "frame-position sink");

// One wave's rows: rollout lr of the launch per 16-lane row (lane j = body j), H steps.  FROW: the
// row after the last rollout is the previous update's filter() (fx0 / fU / fsteps / frec).  The
// costs are not summed here: every step's record goes to HBM and fr_step_cost_kernel evaluates
// the objective for all (rollout, step) pairs at once, a lane each, instead of 16 lanes of a row
// repeating its row-uniform terms.
// HO = 3 (the relay, fr_coop_x_kernel): the call runs steps [kb, ke) only.  kb > 0 resumes from
// the lanes' (q, qd, E) the previous relay stage left in Lst at the top of step kb (the records up
// to it are stored); ke < H - 1 leaves the state there for the next stage.
//
// The relay exists because R + 1 = S + 3 rows of four per wave need one wave more than there are
// SIMDs: at 4096 x 64 the workgroup that holds the rows left over runs them in a fifth wave.  On
// one SIMD beside a main wave the two shared its issue slots for the whole horizon; a single wave
// leaves about 30 % of them idle (one VALU instruction per ~5.6 cycles against ~4 for two waves,
// profiles/r03_ubench.txt), so a second wave with priority takes most of the slots it needs from
// that slack.  The rows therefore travel: relay stage r (wave 4 + r, on SIMD r) runs a quarter of
// the horizon at priority 3 and hands the state to the next stage through LDS, so each of the four
// main waves loses about a quarter of what wave 0 alone lost before.
// PROG: the wave stores its step into *Lprog at the top of each step (the objective chunks, cost_work).
// bound of a relay stage's wait for its state (short sleeps: about 0.2 s)
constexpr int WAIT_SPINS_ROWS = 1 << 22;

// KC: compact records (FR_REC_C, store_ks: the kinematic sums on the row's chain), else the 768-B
// ones (store_kin).
template <int CK, bool EN, bool FROW, int HO = 0, bool PROG = false, bool KC = false>
__device__ __forceinline__ int coop_rows(const FrRolloutArgs &a, int64_t lr, int lane, int wblk, double *Lk, double *Lw,
                                         const double *Lmodel, const double *Lx0, double *Lst = nullptr, int kb = 0,
                                         int ke = 0x7FFFFFFF, int *Lprog = nullptr, int *Lgo = nullptr, int go_val = 0,
                                         RelayXfer *gx = nullptr, int gm = 0)
{
    const int j = lane & (ROW - 1);
#ifdef COOP_TRACE
    if (a.trace && lane == 0 && kb == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.trace[4 * wblk + 0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        a.trace[4 * wblk + 2] = hw;
        a.trace[4 * wblk + 3] = xcc;
    }
#endif
    // FROW: the row after the last rollout is the previous update's filter() (optimal rollout)
    const bool frow = FROW && a.fcost != nullptr && lr == a.count;
    const bool live = lr < a.count || frow;
    if (!live) return -1;   // row-uniform: the row's lanes leave together (no DPP partner is lost)
    const int H = a.H;
    const bool opt_row = a.optimal || frow;   // no noise (mppi.cpp:450-479)
    // U*_shifted row k is Up row min(k + ush, H - 1): with the draws made ahead (a.drawn_ahead) the
    // shift reads U* itself (mppi.cpp:197-207); the state staged in LDS (stage_x0)
    const double *Up = FROW && frow ? a.fU : a.Ushift;
    const int ush = FROW && frow ? 0 : a.ush;
    constexpr int RS = KC ? FR_REC_C : FR_REC;
    double *rp = FROW && frow ? a.frec : a.rec + lr * H * RS;   // [rollout][step][RS]
    auto recp = [&](int k) -> double * { return rp + (int64_t)k * RS; };
    const bool jl = j < FR_NB;   // lane owns a body / control component
    const int jb = jl ? j : 0;
    const double *M = Lmodel + (jl ? j : FR_NB) * MB;
    LaneConst L;
    L.is_rz = jl && FR_KIND[jb] == KIND_RZ;
    {
        double rz = L.is_rz ? 1.0 : 0.0, nrz = 1.0 - rz;
        asm volatile("" : "+v"(rz), "+v"(nrz));   // kept in registers across the loop
        L.rz = rz;
        L.nrz = nrz;
    }
    L.slot = jl ? j : FR_NB;
    L.m_j12 = opaque_mask(j == 12);
    L.m_j13 = opaque_mask(j == 13);
    L.m_j14 = opaque_mask(j == 14);
    L.m_j15 = opaque_mask(j == 15);
    {
        double cA = j == 0 ? 1.0 : 0.0, cB = j == 1 ? 1.0 : 0.0, cC = j == 2 ? 1.0 : 0.0;
        double ck = j > 2 ? 1.0 : 0.0, ct = (j >= 3 && j < 10) ? 1.0 : 0.0;
        asm volatile("" : "+v"(cA), "+v"(cB), "+v"(cC), "+v"(ck), "+v"(ct));   // kept in registers
        L.bA = cA;
        L.bnA = -cA;
        L.bB = cB;
        L.bC = cC;
        L.bkeep = ck;
        L.taud = ct;
    }
    {
        int anc = (1 << (j < 11 ? j : 11)) - 1;   // bodies i < j
        if (j == FR_NB - 1) anc &= ~(1 << (FR_NB - 2));   // finger 11 is not under finger 10
        asm volatile("" : "+v"(anc));
        int ro = j < FR_NB ? 2 * j : REC_E;
        asm volatile("" : "+v"(ro));
        L.rec_off = ro;
        int fo = j == FR_EE_PARENT ? REC_EE : (j == FR_AM_PARENT ? REC_AM : (KC ? REC_SINK_C : REC_FP_SINK));
        asm volatile("" : "+v"(fo));
        L.fp_off = fo;
        if constexpr (KC) {   // store_ks: sum m's x and y in a body slot (S linear 0..2, qd at 3, or 6 with the tank)
            const int m = j < 9 ? j : 8;
            int ka = (int)((0x211000210ull >> (4 * m)) & 0xF);
            int kb = (int)(((EN ? 0x221210666ull : 0x221210333ull) >> (4 * m)) & 0xF);
            asm volatile("" : "+v"(ka), "+v"(kb));   // opaque: the LDS reads stay behind the row's stores
            L.ka = ka;
            L.kb = kb;
            L.m_vsum = opaque_mask(m < 3);
        }
#pragma unroll
        for (int i = 0; i < 10; i++) {
            double d = ((anc >> i) & 1) ? 1.0 : 0.0;
            if (i != 3 && i != 7) asm volatile("" : "+v"(d));   // kept in registers across the loop, not rebuilt per step
            L.ancd[i] = d;
        }
        constexpr int parent[9] = {9, 9, 8, 7, 6, 5, 4, 3, 2};   // of composite_scan's children 11, 10, 9, .., 3
#pragma unroll
        for (int e = 0; e < 9; e++) {
            double d = j == parent[e] ? 1.0 : 0.0;
            asm volatile("" : "+v"(d));   // kept in registers across the loop, not rebuilt per step
            L.cmask[e] = d;
        }
    }
    L.mc = M[T_MC];
    L.inv_m0 = 1.0 / Lmodel[0 * MB + T_MC];   // the base pivots' constant diagonals (gj_pivot_0 / 1)
    L.inv_m1 = 1.0 / Lmodel[1 * MB + T_MC];
    {
        double f0 = j == 0 ? 0.0 : -L.inv_m0, f1 = j == 1 ? 0.0 : -L.inv_m1;
        double qs = j == 0 ? L.inv_m0 : (j == 1 ? L.inv_m1 : 1.0);
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(qs));   // kept in registers across the loop
        L.f0 = f0;
        L.f1 = f1;
        L.qs = qs;
    }

    if (HO != 3) kb = 0;
    const int kend = HO == 3 ? min(ke, H - 1) : H - 1;   // steps [kb, kend) in this call
    // eps and U*_shifted of step k: loaded at the top of the step
    const bool sampled = !opt_row && jl;
    double sd = sampled ? 1.0 : 0.0, jd = jl ? 1.0 : 0.0;
    asm volatile("" : "+v"(sd), "+v"(jd));   // opaque: kept as data, not folded into control flow
    int64_t nstride = sampled ? a.Rpad * FR_C : 0;   // unsampled rows re-read their first element
    asm volatile("" : "+v"(nstride));
    const double *np = sampled ? a.noise + lr * FR_C + jb : Up;   // any valid address when unused
    // eps and U*_shifted one step ahead: the noise tensor streams from HBM / the Infinity Cache,
    // whose latency a single wave per SIMD cannot hide within one step
    // (issued before the first record store: the loop header then waits for the loads alone,
    // vmcnt(2), on the entry edge as on the back edge, not for the stores behind them)
    double eps_n = np[(int64_t)kb * nstride], ub_n = Up[min(kb + ush, H - 1) * FR_C + jb];
    // a relay stage past the first: its setup above and its first loads are in flight while it waits
    // for the previous stage's state (Lgo: the stage counter it raises once Lst is written)
    if constexpr (HO == 3) {
        if (kb > 0 && Lgo != nullptr) {
            int st = 0;
            for (int i = 0; i < WAIT_SPINS_ROWS && st < go_val; i++) {
                st = __builtin_amdgcn_readfirstlane(__hip_atomic_load(Lgo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (st < go_val) __builtin_amdgcn_s_sleep(1);
            }
            asm volatile("" ::: "memory");   // the reads of Lst below stay behind the poll (LDS is in order)
            if (st < go_val) {
                if (lane == 0) {
                    if (a.status) atomicAdd(&const_cast<Status *>(a.status)->wait_timeouts, 1);
                    if (a.wait_sum) atomicAdd(a.wait_sum, 1.0);
                }
                return -2;   // (the stage never ran)
            }
        }
    }
    double q, qd, E;
    if (HO == 3 && gx != nullptr) {   // a later relay member's first stage: the previous member's state
        bool ok = false;                // (the launch's token, then sc1 loads; bounded, -2 if it gave up)
        for (int i = 0; i < WAIT_SPINS_ROWS && !ok; i++) {
            ok = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&gx->state_tok[gm - 1][0], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT)) == a.rtoken;
            if (!ok) __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) {
            if (lane == 0) {
                if (a.status) atomicAdd(&const_cast<Status *>(a.status)->wait_timeouts, 1);
                if (a.wait_sum) atomicAdd(a.wait_sum, 1.0);
            }
            return -2;
        }
        q = __hip_atomic_load(&gx->state[gm - 1][3 * lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qd = __hip_atomic_load(&gx->state[gm - 1][3 * lane + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        E = __hip_atomic_load(&gx->state[gm - 1][3 * lane + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (kb > 0) {   // the state the previous relay stage left at the top of step kb
        q = Lst[3 * lane];
        qd = Lst[3 * lane + 1];
        E = Lst[3 * lane + 2];
    } else {
        // the folded filter() row's state from global memory, the update's from LDS: values
        // selected, not pointers (a select of the two is a generic pointer, whose loads leave the
        // step loop's header waiting for every store in flight, vmcnt(0))
        double fq = 0.0, fqd = 0.0, fE = 0.0;
        if (FROW && frow) {
            fq = a.fx0[jb];
            fqd = a.fx0[FR_NB + jb];
            fE = EN ? a.fx0[FR_X - 1] : 0.0;
        }
        const double lq = Lx0[jb], lqd = Lx0[FR_NB + jb], lE = EN ? Lx0[FR_X - 1] : 0.0;
        q = jl ? (FROW && frow ? fq : lq) : 0.0;
        qd = jl ? (FROW && frow ? fqd : lqd) : 0.0;
        E = EN ? (FROW && frow ? fE : lE) : 0.0;   // EnergyTank::set_energy(state.available_energy)
    }
    const double *grav = a.model->gravity;
    // REGTAB: the body-table fields the step reads, held in registers across the loop instead of
    // re-read from LDS every step (A/B: the loop's VGPR budget against sixteen ds_read2 per step)
    // the fields in REGTAB_MASK (bit n: field n) are loaded once, opaque, and stay in registers; the
    // step's other fields are re-read from LDS in every step (tab_refresh).  Not in the energy-tank
    // kernels, whose registers are spent already (their spills went 13 -> 33 with it).
#ifdef REGTAB
#ifndef REGTAB_MASK
#define REGTAB_MASK 0xFFFFFFFFFFFFull
#endif
    constexpr bool RT = !EN;
#else
#define REGTAB_MASK 0ull
    constexpr bool RT = false;
#endif
    constexpr uint64_t RT_USED = 0x1401FFFFFEDBull;   // fields the step reads (T_R cols 0, 1 .. T_NROT, T_FIX, T_IL)
    double Mreg[T_IL + 1];
    if constexpr (RT) {
#pragma unroll
        for (int n = 0; n <= T_IL; n++) {
            if ((RT_USED >> n) & (REGTAB_MASK >> n) & 1) {
                double v = M[n];
                asm volatile("" : "+v"(v));
                Mreg[n] = v;
            }
        }
    }
    auto tab_refresh = [&]() {
        if constexpr (RT) {
#pragma unroll
            for (int n = 0; n <= T_IL; n++)
                if (((RT_USED >> n) & 1) && !((REGTAB_MASK >> n) & 1)) Mreg[n] = M[n];
        }
    };
    const double *Mk = RT ? Mreg : M;
    double sq, cq;
    const SinCosK scK = sincos_constants();
    fsincos(q, &sq, &cq, scK);   // one sincos per lane and step: FK and base yaw
    CoopKin kin;
    CoopBody bd;
    // coop_solve's block rows: slots 13..15 hold zeros for good (slot 12 is tau, rewritten per step)
    if constexpr (!EN) {
        *reinterpret_cast<double2 *>(Lk + L_COL + j * CSTR + 12) = double2{0.0, 0.0};   // (12: tau with GJ_COLS)
        *reinterpret_cast<double2 *>(Lk + L_COL + j * CSTR + 14) = double2{0.0, 0.0};
        *reinterpret_cast<double2 *>(Lk + L_TP + 12) = double2{0.0, 1.0};   // coop_solve's dummy-lane reads
    }
    if (kb == 0) {
        coop_fk<CK, false>(L, q, sq, cq, qd, M, Lk, kin, bd, grav);   // set_state -> calculate() at (q0, v0)
        if constexpr (KC) store_ks<CK, EN, false>(recp(0), j, L, bd, qd, Lk);   // (coop_fk<CK, false> staged nothing)
        else store_kin<CK>(recp(0), j, bd, qd);
    }

    if (kb == 0) store_record<EN>(recp(0), j, L, q, qd, kin, E);
    // a relay stage enters its loop with nothing in flight (its first step needs step kb's loads
    // anyway): where the entry edge held an unknown count, the loop header waited for every store
    // in flight on every step, the back edge's record stores included
    if constexpr (HO == 3) __builtin_amdgcn_s_waitcnt(0);
    for (int k = kb; k < kend; k++) {
        PMARK(0);
        if constexpr (PROG) __hip_atomic_store(Lprog, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const double eps_l = eps_n, ub_l = ub_n;
        eps_n = np[(int64_t)(k + 1) * nstride];
        ub_n = Up[min(k + 1 + ush, H - 1) * FR_C + jb];
        // u = U*_shifted + eps as data (1.0 / 0.0 coefficients, not selects: a select here became a
        // branch around the eps use, and the waitcnt pass then waited for every store in flight,
        // vmcnt(0), at the top of each step); unsampled rows add 0 eps, lanes 12..15 hold u = 0
        // PinocchioDynamics::step: base velocity overwrite, tau = arm controls, calculate, Euler
        const double u = __builtin_fma(eps_l, sd, ub_l * jd);
        qd = base_velocity(L, u, sq, cq, qd);
        if constexpr (EN)
            Lw[L_TAU + j] = (j >= 3 && j < 10) ? u : 0.0;   // coop_aba's tau
        tab_refresh();
        coop_fk<CK, EN>(L, q, sq, cq, qd, Mk, Lk, kin, bd, grav);
        // the next record's kinematics (the one-step lag)
        if constexpr (KC) store_ks<CK, EN>(recp(k + 1), j, L, bd, qd, Lk);
        else store_kin<CK>(recp(k + 1), j, bd, qd);
        double pe = 0.0;
        double qdd;
        if constexpr (EN) qdd = coop_aba<EN>(j, Lk, Lw, pe);
        else qdd = coop_solve(j, L, bd, u * L.taud, Lk);
        PMARK_D(7, qdd);
        qd = qd + qdd * a.dt;
        q = q + qd * a.dt;
        if constexpr (EN) {   // power = (tau_u + NLE) . v_new; EnergyTank::step (energy.hpp:19-22)
            const double tau_l = (j >= 3 && j < 10) ? u : 0.0;
            const double power = bsum<0, FR_NB>(tau_l * qd + kin.pw, 1.0) + a.dt * bsum<0, 6>(pe, 1.0);
            E = smax(0.0, E + power * a.dt);
        }
        store_record<EN>(recp(k + 1), j, L, q, qd, kin, E);
        PMARK(1);
        fsincos(q, &sq, &cq, scK);
    }
    if (HO == 3 && kend < H - 1) {   // the next relay stage resumes at step kend
        Lst[3 * lane] = q;
        Lst[3 * lane + 1] = qd;
        Lst[3 * lane + 2] = E;
    }
    // the final step's dynamics are never observed (deviation 5)
#ifdef COOP_TRACE
    if (a.trace && lane == 0) a.trace[4 * wblk + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
    return -1;
}

// ---- the objective inside the launch (a.costs_in_launch) ----------------------------------------
// With R + 1 = S + 3 rows on 4S / 16 SIMDs one SIMD runs the fifth wave beside a main wave, and
// every other SIMD idles for the last third of the launch while those two finish.  The objective
// of the rows (fr_cost_terms.hpp rollout_cost: a pass per rollout, lane = step) runs there: each
// main wave evaluates its own rows after its horizon loop, except the fifth wave's SIMD-mate, whose
// rows - and then the fifth wave's - waves 1..3 of the workgroup evaluate once those waves signal
// their records stored (an LDS flag each), so nothing is added to the doubled SIMD.  The per-joint
// parameters are the body table's T_LO .. T_VW fields (stride MB).

// J of local rollout lr (or the folded filter() row) from its records, written out
template <int CK, bool EN, bool KC>
__device__ __forceinline__ void launch_row_cost(const FrRolloutArgs &a, int64_t lr, int lane, const double *Lmodel)
{
    const bool frow = a.fcost != nullptr && lr == a.count;
    if (!(lr < a.count || frow)) return;
    if (frow && (a.status->all_nan || a.status->sg_error)) return;   // no filter() when the update threw
    const double J = mppi_cost::rollout_cost<CK, EN, MB, KC>(*a.cost, frow ? a.fsteps : a.steps,
                                                              frow ? a.frec : a.rec + lr * a.H * (KC ? FR_REC_C : FR_REC), a.H,
                                                              lane, Lmodel + T_LO);
    if (lane == 0) {
        if (frow) *a.fcost = J;
        else {
            a.cost_out[a.begin + lr] = J;
            mppi_cost::fold_cost_stats(a.stats, J, lr);
        }
    }
}

// This wave's record stores are complete and visible to the workgroup; then raise the flag
__device__ __forceinline__ void signal_records(int *flag)
{
    __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the same, one count of several (the relay's stages: Lflag[LF_RELAY] counts those done)
__device__ __forceinline__ void signal_records_add(int *flag)
{
    __builtin_amdgcn_s_waitcnt(0);
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Bounded: a wave that never signals (a bug) costs about a second, not a hung GPU.  The timeout is
// counted in Status::wait_timeouts (and, sharded over RCCL, in the rank's cost slot R that the
// engine all-reduces); the finish kernel then fails the update (MPPI_ERR_DEVICE) instead of
// publishing U* from costs some rows never wrote (kernels.hip update_wait_timeouts).
constexpr int WAIT_SPINS = 1 << 20;
__device__ __forceinline__ void note_wait_timeout(const FrRolloutArgs &a)
{
    if (a.status) atomicAdd(&const_cast<Status *>(a.status)->wait_timeouts, 1);
    if (a.wait_sum) atomicAdd(a.wait_sum, 1.0);
}
__device__ __forceinline__ void wait_records(const FrRolloutArgs &a, int *flag)
{
    // the flag read through readfirstlane: a uniform (scalar-branch) loop whatever the exec mask
    for (int i = 0; i < WAIT_SPINS; i++) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0)
            return;
        __builtin_amdgcn_s_sleep(8);
    }
    if ((threadIdx.x & 63) == 0) note_wait_timeout(a);
}
// The relay's wait across workgroups: until a token word holds this launch's token (a.rtoken).  The
// producer stores its payload sc1 (agent-scope relaxed stores), waits for every one of them
// (s_waitcnt 0), then one lane stores the token sc1; this wave polls with sc1 loads and loads the
// payload with sc1 loads after the match (MI355X_MICROARCH.md, inter-workgroup visibility: one
// storing wave, sc1 both sides, the polling wave loads).  Bounded; returns whether it arrived.
__device__ __forceinline__ bool wait_token(const FrRolloutArgs &a, uint32_t *word)
{
    for (int i = 0; i < WAIT_SPINS; i++) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == a.rtoken)
            return true;
        __builtin_amdgcn_s_sleep(4);
    }
    if ((threadIdx.x & 63) == 0) note_wait_timeout(a);
    return false;
}

// the same bounded wait, returning the value it saw (0 if it gave up)
__device__ __forceinline__ int wait_nonzero(const FrRolloutArgs &a, int *word)
{
    for (int i = 0; i < WAIT_SPINS; i++) {
        const int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (v != 0) return v;
        __builtin_amdgcn_s_sleep(8);
    }
    if ((threadIdx.x & 63) == 0) note_wait_timeout(a);
    return 0;
}

// The next update's draws for the wave's own four rows (a.ahead_noise), made in the launch's idle
// tail after the rows' objective: draw_ahead_block's values (Philox by (rollout, step) with the
// next update's index, Box-Muller, the diagonal transform), rows of rollouts >= 2 only.  Lane
// items run step-major over (row, piece), so twelve consecutive lanes store one step's 384
// contiguous bytes.  The wave read its rows' previous eps (kept columns) at entry, so the buffer
// is free; no other wave touches these rows.
__device__ __forceinline__ void tail_draws(const FrRolloutArgs &a, int64_t lr0, int lane)
{
    const SampleArgs &sa = a.samp;
    const int H = sa.H;
    const uint32_t upd = (uint32_t)(sa.sp.update_index + 1);
    const uint32_t s0 = (uint32_t)sa.sp.seed, s1 = (uint32_t)((uint64_t)sa.sp.seed >> 32);
#pragma unroll 1
    for (int it = lane; it < 12 * H; it += 64) {
        const int blk = it % 3, i = (it / 3) % 4, k = it / 12;
        const int64_t lr = lr0 + i, g = sa.begin + lr;
        if (lr >= sa.count || g < 2) continue;
        const int64_t draw = mppi_sample::philox_index(g, k, H);
        const mppi_dev::u32x4 ctr{(uint32_t)draw, (uint32_t)((uint64_t)draw >> 32), upd, (uint32_t)blk};
        const mppi_dev::u32x4 r = mppi_dev::philox4x32_10(ctr, s0, s1);
        float z[4];
        mppi_dev::box_muller(r.x, r.y, z[0], z[1]);
        mppi_dev::box_muller(r.z, r.w, z[2], z[3]);
        double2 *o = reinterpret_cast<double2 *>(a.ahead_noise + ((int64_t)k * sa.Rpad + lr) * FR_C + 4 * blk);
        o[0] = double2{sa.tdv[4 * blk] * (double)z[0], sa.tdv[4 * blk + 1] * (double)z[1]};
        o[1] = double2{sa.tdv[4 * blk + 2] * (double)z[2], sa.tdv[4 * blk + 3] * (double)z[3]};
    }
}

// Whether launch row lr exists (a rollout of the shard or the folded filter() row)
__device__ __forceinline__ bool row_live(const FrRolloutArgs &a, int64_t lr)
{
    return lr < a.count || (a.fcost != nullptr && lr == a.count);
}

// ---- the objective in chunks, beside the horizon loops (fr_coop_x_kernel) ----------------------
// One wave per SIMD leaves about 30 % of its issue slots idle (r03_ubench).  fr_coop_x_kernel fills
// them with a second wave per SIMD that evaluates the objective while the rows still run: the step
// costs of a row group (a main wave's four rows, or the relay's) in chunks of CH steps, lane =
// (row, step), as soon as the chunk's records are stored.  Those waves run at priority 0, the main
// waves at 1.  Each chunk's 64 step costs go to LDS (Lcs); the wave that completes a group's last
// chunk sums every row's step costs in step order (the reference's J += cost, mppi.cpp:322-337:
// the same additions as rollout_cost) and writes J.  A main wave stores its loop step into LDS
// (Lq[Q_PROG + g]) at the top of every step.  Seeing step p there means the wave has waited, in
// step p - 1, for the eps loads it issued in step p - 2 after storing record p - 2; vector memory
// operations complete in order on gfx9 (one vmcnt for loads and stores), so records up to p - 2
// are complete.  A chunk is taken when records up to its last are complete with a step to spare
// (p >= last + 3), and the last chunk after the wave's loop (its flag, behind s_waitcnt 0).  Chunks
// of CH = 16 records are whole 128-byte lines (16 x 336 B = 42 lines, rows 21504 B apart), so no
// line a chunk reads is written after it.  The relay's rows are taken after their last stage.
constexpr int CH = 16;          // steps per chunk
constexpr int HC_MAX = 128;     // the horizon bound of the objective in this launch (Lcs)
// LDS words (Lq): the main waves' steps, the groups' next chunk to take and chunks completed, the
// relay's stage
enum { Q_PROG = 0, Q_NEXT = 4, Q_DONE = 9, Q_STAGE = 14, Q_N = 16 };
// LDS flags (Lflag): main wave g's records are stored (g), the relay's rows are done (LF_RELAY),
// main wave g's kept columns are copied (LF_KEPT + g: its rows' previous eps is read, so their next
// draws may overwrite it)
constexpr int LF_RELAY = 4, LF_KEPT = 5, LF_KEPT_X = 9, LF_N = 10;   // LF_KEPT_X: the relay rows' kept columns are copied

__device__ __forceinline__ int lds_read(int *w)
{
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// The relay over a.relay_k workgroups: relay group q (rows [xbase + 4 q, xbase + 4 q + 4)) runs in
// workgroups q + RELAY_STRIDE m, m < relay_k (one XCD under the dispatcher's round-robin placement:
// speed only, nothing relies on it), member m over chunks [m nch / K, (m + 1) nch / K) of the horizon
// - the records member m stores are the ones it evaluates.  -1: the workgroup holds no relay rows.
__device__ __forceinline__ int relay_member(const FrRolloutArgs &a)
{
    const int nxb = (int)((a.xrows + ROWS_PER_WAVE - 1) / ROWS_PER_WAVE);
    const int q = (int)blockIdx.x % RELAY_STRIDE, m = (int)blockIdx.x / RELAY_STRIDE;
    return (q < nxb && m < a.relay_k) ? m : -1;
}
// member m's first loop step: 0, else the step that stores the first record of its first chunk
__device__ __forceinline__ int relay_member_step(const FrRolloutArgs &a, int m, int H)
{
    if (m <= 0) return 0;
    if (m >= a.relay_k) return H - 1;
    return (m * ((H + CH - 1) / CH) / a.relay_k) * CH - 1;
}
// first launch row of group g (main wave g of the workgroup, or the relay's rows for g = 4)
__device__ __forceinline__ int64_t group_row0(const FrRolloutArgs &a, int g)
{
    return g < 4 ? ((int64_t)blockIdx.x * 4 + g) * ROWS_PER_WAVE
                 : a.xbase + (int64_t)((int)blockIdx.x % RELAY_STRIDE) * ROWS_PER_WAVE;
}
// the chunks [c0, c1) of group g this workgroup evaluates: a main wave's every chunk; of the relay's
// rows, its member's share
__device__ __forceinline__ void group_chunks(const FrRolloutArgs &a, int g, int &c0, int &c1)
{
    const int nch = (a.H + CH - 1) / CH;
    c0 = 0;
    c1 = nch;
    if (g == 4 && a.relay_k > 1) {
        const int m = (int)blockIdx.x / RELAY_STRIDE;
        c0 = m * nch / a.relay_k;
        c1 = (m + 1) * nch / a.relay_k;
    }
}
// whether chunk c of group g can be read: its records are complete
__device__ __forceinline__ bool chunk_ready(const FrRolloutArgs &a, int g, int c, int *Lflag, int *Lq)
{
    if (g == 4) return lds_read(Lflag + LF_RELAY) >= (a.handover ? 4 : 1);   // every stage here has stored its records
    const int last = min((c + 1) * CH, a.H) - 1;
    if (last < a.H - 1 && lds_read(Lq + Q_PROG + g) >= last + 3) return true;
    return lds_read(Lflag + g) != 0;
}

// The step costs of chunk c of group g into Lcs; the pass that completes the group sums its rows
template <int CK, bool EN>
__device__ __forceinline__ void cost_chunk(const FrRolloutArgs &a, int g, int c, int lane, const double *Lmodel, double *Lcs,
                                          int *Lq)
{
    const int H = a.H;
    int cb, ce;
    group_chunks(a, g, cb, ce);   // the group's chunks in this workgroup
    const int i = lane >> 4, k = c * CH + (lane & 15);
    const int64_t lr0 = group_row0(a, g), lr = lr0 + i;
    const bool rl = row_live(a, lr), live = rl && k < H;
    const bool frow = a.fcost != nullptr && lr == a.count;
    const int64_t lrv = rl ? lr : lr0;   // any live row's records when unused
    const double *rec = frow ? a.frec : a.rec + lrv * H * FR_REC;
    const StepConst *stp = frow ? a.fsteps : a.steps;
    const int kk = live ? k : 0;
    PMARK(8);
#ifndef COST_JG
#define COST_JG 2
#endif
    double cs = mppi_cost::record_step_cost<CK, EN, MB, false, COST_JG>(*a.cost, stp[kk], rec + (int64_t)kk * FR_REC, Lmodel + T_LO);
    PMARK_D(9, cs);
    if (live) Lcs[(g * ROWS_PER_WAVE + i) * HC_MAX + k] = cs;
    // the stores before the count: the wave that completes the group reads every chunk's costs
    const int n = __builtin_amdgcn_readfirstlane(
        __hip_atomic_fetch_add(Lq + Q_DONE + g, lane == 0 ? 1 : 0, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (n + 1 != ce - cb) return;
    // the relay's rows over several workgroups: the partial sums arrive from the previous member and
    // go on to the next (the reference's J += cost in step order across the members)
    const int m = (int)blockIdx.x / RELAY_STRIDE;
    const bool from_prev = g == 4 && a.relay_k > 1 && m > 0;
    const bool to_next = g == 4 && a.relay_k > 1 && m + 1 < a.relay_k;
    RelayXfer *x = (from_prev || to_next) ? a.rx + ((int)blockIdx.x % RELAY_STRIDE) : nullptr;
    double J0 = 0.0;
    if (from_prev) {   // bounded; on a timeout the update fails (wait_timeouts)
        const bool ok = wait_token(a, &x->sums_tok[m - 1][0]);
        J0 = (ok && lane < ROWS_PER_WAVE) ? __hip_atomic_load(&x->sums[m - 1][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    }
    if (lane < ROWS_PER_WAVE) {
        const int64_t r = lr0 + lane;
        if (row_live(a, r) || to_next) {
            const double *cr = Lcs + (g * ROWS_PER_WAVE + lane) * HC_MAX;
            // J += c_q in step order, the loads sixteen at a time: one LDS round trip per sixteen
            // adds, not per add (the one-by-one loop waited on every ds_read: ~3 us at the end of
            // every workgroup's last chunk)
            double J = J0;
            const int Hend = min(ce * CH, H);
            int q = cb * CH;
            for (; q + 16 <= Hend; q += 16) {
                double c[16];
#pragma unroll
                for (int u = 0; u < 16; u += 2) {
                    const double2 v = *reinterpret_cast<const double2 *>(cr + q + u);
                    c[u] = v.x;
                    c[u + 1] = v.y;
                }
#pragma unroll
                for (int u = 0; u < 16; u++) J += c[u];
            }
            for (; q < Hend; q++) J += cr[q];
            if (to_next) {   // the next member continues from these (sc1, then the token)
                __hip_atomic_store(&x->sums[m][lane], J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_s_waitcnt(0);
                if (lane == 0) __hip_atomic_store(&x->sums_tok[m][0], a.rtoken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            J = isnan(J) ? (double)NAN : J;
            if (a.fcost != nullptr && r == a.count) {
                if (!(a.status->all_nan || a.status->sg_error)) *a.fcost = J;   // no filter() when the update threw
            } else {
                a.cost_out[a.begin + r] = J;
                mppi_cost::fold_cost_stats(a.stats, J, r);
            }
        }
    }
}

// A wave's objective work: chunks of any group, its own group (first) first, each taken from the
// group's counter when it is ready (a chunk taken just as another wave took the one before it
// waits for its records); returns once every chunk is taken.  Bounded.
template <int CK, bool EN>
__device__ __forceinline__ void cost_work(const FrRolloutArgs &a, int first, int ng, int lane, const double *Lmodel,
                                         double *Lcs, int *Lflag, int *Lq)
{
#pragma unroll 1
    for (int spin = 0; spin < WAIT_SPINS; spin++) {
        bool left = false, did = false;
#pragma unroll 1
        for (int d = 0; d < ng && !did; d++) {
            const int g = first + d < ng ? first + d : first + d - ng;
            int cb, nch;
            group_chunks(a, g, cb, nch);   // (Lq[Q_NEXT + g] starts at cb)
            const int c0 = lds_read(Lq + Q_NEXT + g);
            if (c0 >= nch) continue;
            left = true;
            if (!chunk_ready(a, g, c0, Lflag, Lq)) continue;
            // every lane executes the add (lane 0 adds 1): no lane-dependent branch around it
            const int c = __builtin_amdgcn_readfirstlane(
                __hip_atomic_fetch_add(Lq + Q_NEXT + g, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (c >= nch) continue;
            int w = 0;
            while (!chunk_ready(a, g, c, Lflag, Lq) && w < WAIT_SPINS) {
                __builtin_amdgcn_s_sleep(4);
                w++;
            }
            if (w == WAIT_SPINS && lane == 0) note_wait_timeout(a);
#ifdef COST_TRACE   // block 0's chunks: start, end, wave (slots past the relay's)
            const uint32_t tc0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
            cost_chunk<CK, EN>(a, g, c, lane, Lmodel, Lcs, Lq);
#ifdef COST_TRACE
            if (a.trace && blockIdx.x == 0 && lane == 0 && c < 4) {
                uint32_t *tr = a.trace + 4 * (gridDim.x * 4 + 16 + 4 * g + c);
                tr[0] = tc0;
                tr[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                tr[2] = threadIdx.x >> 6;
            }
#endif
            did = true;
        }
        if (!left) return;
        if (!did) __builtin_amdgcn_s_sleep(8);
    }
    if (lane == 0) note_wait_timeout(a);
}

// The next update's draws for main wave g's rows, once its kept columns are copied
__device__ __forceinline__ void group_draws(const FrRolloutArgs &a, int g, int lane, int *Lflag)
{
    wait_records(a, Lflag + LF_KEPT + g);
    tail_draws(a, group_row0(a, g), lane);
}

// fr_coop_kernel's four-wave launch (no rows left over): each main wave evaluates its own rows'
// objective after its loop (rollout_cost, a pass per row, lane = step) and makes their next draws
template <int CK, bool EN, bool KC>
__device__ __forceinline__ void launch_costs(const FrRolloutArgs &a, int wv, int lane, const double *Lmodel)
{
    const int64_t w0 = (int64_t)blockIdx.x * 4;
    __builtin_amdgcn_s_waitcnt(0);   // the wave's own record stores, read back by other lanes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
    for (int i = 0; i < ROWS_PER_WAVE; i++) launch_row_cost<CK, EN, KC>(a, (w0 + wv) * ROWS_PER_WAVE + i, lane, Lmodel);
    if (a.ahead_noise) tail_draws(a, (w0 + wv) * ROWS_PER_WAVE, lane);
}

// Relay stage r's steps [relay_step(r), relay_step(r + 1)): member m = r / 4 of the relay runs stages
// 4 m .. 4 m + 3, quarters of its steps; one member: quarters of the H - 1 loop steps
__device__ __forceinline__ int relay_step(const FrRolloutArgs &a, int r, int H)
{
    if (r >= 4 * a.relay_k) return H - 1;
    const int m = r / 4, k0 = relay_member_step(a, m, H), k1 = relay_member_step(a, m + 1, H);
    return k0 + ((r % 4) * (k1 - k0)) / 4;
}

// Relay stage s (wave 4 + s) of member m of a relay group (a.handover): makes the next update's draws
// for main wave s's rows (but main wave 0's of member 0, which rank_draw_kernel makes, as the engine
// expects of the first wave of these workgroups), waits for stage s - 1 (Lq[Q_STAGE] == s) - or, as
// a later member's first stage, for the previous member's state (rx, sc1, the launch's token) -
// runs its part of the horizon at priority 3 and passes the state on; each member's last stage
// raises its workgroup's relay records flag.  With relay_k members every SIMD that hosts a stage
// carries 1 / (4 relay_k) of the extra wave instead of a quarter (the host main waves lost ~20 us
// each to their stage with one member, r06 wave traces); the stages' loop is the same code, only the
// hand-off crosses workgroups, once per member.  Without a.handover wave 4 runs every step itself
// at the main waves' priority (the doubled SIMD of round 2, kept for A/B).  Returns whether the
// stage ran (false: the previous stage never signalled, counted in Status::wait_timeouts).
template <int CK, bool EN>
__device__ __forceinline__ bool relay_stage(const FrRolloutArgs &a, int s, int m, int lane, double *Lk, double *Lw,
                                            const double *Lmodel, const double *Lx0, int *Lflag, int *Lq, double *Lst)
{
    const int H = a.H;
    const int q = (int)blockIdx.x % RELAY_STRIDE;
    const int64_t xlr = a.xbase + (int64_t)q * ROWS_PER_WAVE + (lane >> 4);
    const int wblk = gridDim.x * 4 + q;   // (the relay rows' trace slot)
    const int r = 4 * m + s;
    int kb = 0, ke = 0x7FFFFFFF;   // without a.handover: every step on this wave (one stage)
    if (a.handover) {
        // the next update's draws for main wave s's rows (member 0's wave 0 rows are left to
        // rank_draw_kernel): first where the stage waits long for its turn (later members), after
        // the stage in member 0, whose stages follow each other within microseconds when the relay
        // spans several workgroups
        if (m > 0 && a.ahead_noise) group_draws(a, s, lane, Lflag);
        __builtin_amdgcn_s_setprio(3);   // above the main waves (1) and the objective's (0)
        kb = relay_step(a, r, H);
        ke = relay_step(a, r + 1, H);
    }
    // a stage past the first issues its first eps loads before it waits for the previous stage: the
    // relay rows' kept columns (wave 4's copy at entry, this member's steps) must have landed
    if (s > 0 && a.drawn_ahead) wait_records(a, Lflag + LF_KEPT_X);
    // one call site: one copy of the step loop for both shapes.  A stage past a member's first makes
    // its setup and first loads, then waits inside for the previous stage's state (Lq[Q_STAGE] == s;
    // bounded, about 0.2 s: -2 if it gave up)
    if (coop_rows<CK, EN, true, 3>(a, xlr, lane, wblk, Lk, Lw, Lmodel, Lx0, Lst, kb, ke, nullptr,
                                   (a.handover && s > 0) ? Lq + Q_STAGE : nullptr, s,
                                   (a.handover && s == 0 && m > 0) ? a.rx + q : nullptr, m) == -2)
        return false;
    if (a.handover) {
        __builtin_amdgcn_s_setprio(0);
#ifdef COOP_TRACE   // the stages' ends of relay group 0, member m in the slot 1 + m past the relay rows'
        if (a.trace && q == 0 && lane == 0) a.trace[4 * (gridDim.x * 4 + 1 + m) + s] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
        if (s < 3) {   // the state in Lst (LDS) is all the next stage waits for: signal it at once
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // fault injection (tests only): stage 1 never signals, so stages 2 and 3 time out
            if (!((a.debug & 1) && r == 1))
                __hip_atomic_store(Lq + Q_STAGE, s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // then this stage's record stores, counted for the relay's cost chunks
            if (a.costs_in_launch) signal_records_add(Lflag + LF_RELAY);
            if (m == 0 && s > 0 && a.ahead_noise) group_draws(a, s, lane, Lflag);   // (member 0: after the stage)
            return true;
        }
        if (m + 1 < a.relay_k) {   // the last stage of a member: the state to the next member (sc1), then the token
            RelayXfer *x = a.rx + q;
#pragma unroll
            for (int c = 0; c < 3; c++)
                __hip_atomic_store(&x->state[m][3 * lane + c], Lst[3 * lane + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) __hip_atomic_store(&x->state_tok[m][0], a.rtoken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (blockIdx.x == 0 && lane == 0) const_cast<Status *>(a.status)->handover = a.handover ? relay_step(a, 1, H) : -1;
    if (a.costs_in_launch) signal_records_add(Lflag + LF_RELAY);   // this workgroup's relay records are stored
    if (a.handover && m == 0 && s > 0 && a.ahead_noise) group_draws(a, s, lane, Lflag);   // (member 0: after the stage)
    return true;
}

// The update's state into LDS: from the launch's arguments with the draws made ahead, else from x0
__device__ __forceinline__ void stage_x0(const FrRolloutArgs &a, double *Lx0)
{
    if ((int)threadIdx.x < MAX_X) {   // (values selected, not pointers: a select of the argument block and a
                                      // global pointer is a generic pointer, whose load waits on LDS too)
        const double va = a.samp.x0v[threadIdx.x], vx = a.x0[threadIdx.x < FR_X ? threadIdx.x : 0];
        Lx0[threadIdx.x] = a.drawn_ahead ? va : vx;
    }
}

// Draws ahead (a.drawn_ahead): the eps tensor already holds this update's draws, made by
// draw_ahead_kernel behind the previous update; only the kept rollouts' columns from the previous
// eps remain (rank < keep: steps k < shifted, or every step when nothing shifted).  A wave copies
// its own kept rows before its horizon loop (rk: the row's rank, loaded at kernel entry so the load
// overlaps the table staging), lanes 0..11 of a row = 3 pieces x 4 step phases, loads of UN steps
// in flight before their stores.  Waves without a kept row start at once.
__device__ __forceinline__ int kept_rank(const FrRolloutArgs &a, int64_t lr)
{
    const int64_t g = a.samp.begin + lr;
    return (a.drawn_ahead && lr < a.count && g >= 2) ? a.samp.rank[g] : 0x7FFFFFFF;
}
// [kmin, kmax): the steps whose columns this wave copies (a relay member: the steps it runs)
__device__ __forceinline__ void kept_rows_wave(const FrRolloutArgs &a, int64_t lr, int lane, int rk, int kmin = 0,
                                               int kmax = 0x7FFFFFFF)
{
    const SampleArgs &sa = a.samp;
    const bool kept = rk < sa.sp.keep;
    if (__ballot(kept) == 0) return;
    const int j = lane & 15;
    if (kept && j < 12) {
        const int blk = j % 3, ph = j / 3;
        const int kend = min(sa.sp.shift_by > 0 ? (int)sa.sp.shifted : sa.H, kmax);
        const int kst = kmin <= ph ? ph : ph + ((kmin - ph + 3) / 4) * 4;   // the first step >= kmin of this phase
        const int64_t sh = sa.sp.shift_by > 0 ? sa.sp.shift_by : 0;
        constexpr int UN = 8;
        typedef double d2v __attribute__((ext_vector_type(2)));   // (HIP's double2 kept v on the stack)
        for (int k0 = kst; k0 < kend; k0 += 4 * UN) {
            d2v v[UN][2];
#pragma unroll
            for (int u = 0; u < UN; u++) {
                const int k = k0 + 4 * u < kend ? k0 + 4 * u : kst;
                const d2v *src = reinterpret_cast<const d2v *>(sa.prev + (((int64_t)k + sh) * sa.Rpad + lr) * FR_C + 4 * blk);
                v[u][0] = src[0];
                v[u][1] = src[1];
            }
            // past kend the loads read step kst's source and the stores rewrite step kst with it (the
            // value its first store wrote): no branch per store, so v stays in registers (a
            // conditional store sequence put it on the stack)
#pragma unroll
            for (int u = 0; u < UN; u++) {
                const int k = k0 + 4 * u < kend ? k0 + 4 * u : kst;
                double *dst = sa.noise + ((int64_t)k * sa.Rpad + lr) * FR_C + 4 * blk;
                reinterpret_cast<d2v *>(dst)[0] = v[u][0];
                reinterpret_cast<d2v *>(dst)[1] = v[u][1];
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);   // the copies land before the row's lanes read them
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// Block 0's share of sampling in draws-ahead launches: U*_shifted and x0 written back for
// the kernels after the launch.  (The cost statistics the rows fold into were reset by the previous
// update's finish kernel, a launch ahead: no reset races the folds inside this launch.)
template <int NT>
__device__ __forceinline__ void block0_sample_writes(const FrRolloutArgs &a, int t)
{
    const SampleArgs &sa = a.samp;
    if (sa.sp.shift_by > 0)
        for (int i = t; i < sa.H * FR_C; i += NT) sa.Us[i] = mppi_sample::shifted_u(sa, i / FR_C, i % FR_C);
    if (t < sa.X) sa.x0_out[t] = sa.x0v[t];
}

// WPB waves per workgroup.  The update's launch uses WPB = 5 with > 80 KB of LDS per workgroup, so a
// CU holds one workgroup: waves 0..3 take one SIMD each, and wave 4 runs the rows left over when
// the rollouts do not fill four-wave groups (rollouts 0 and 1 of the reference's R = S + 2, plus the
// previous update's filter()) or exits at once.  With one-wave workgroups the dispatcher balances
// waves per CU but not per SIMD: the ~9 % of SIMDs it gave two waves ran 1.23x longer and set the
// kernel's time, and a separate launch for the leftover rows was placed by XCD round-robin, not
// on the free CU (per-block traces, tools/wave_trace.py).
// KC: compact records with the kinematic sums on the rows' chains (the update's launches, throughput-
// bound); the standalone filter() row (one latency-bound row) keeps the 768-B record and a shorter step.
template <int CK, bool EN, int WPB, bool FROW, bool KC>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(2, 2))) void fr_coop_kernel(FrRolloutArgs a)
{
    constexpr int KS = EN ? LDS_KIN_EN : LDS_KIN;
    __shared__ __attribute__((aligned(16))) double lds_kin[WPB * ROWS_PER_WAVE * KS];
    __shared__ __attribute__((aligned(16))) double lds_scr[WPB * ROWS_PER_WAVE * LDS_SCR];
    __shared__ double Lmodel[LDS_MODEL];
    __shared__ double Lx0[MAX_X];
    if (a.optimal && (a.status->all_nan || a.status->sg_error)) return;   // no filter() (mppi.cpp:170-176)
    const int wv = (WPB == 1) ? 0 : (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int rowi = lane >> 4;
    const int wrow = wv * ROWS_PER_WAVE + rowi;   // row within the workgroup
    const int wblk = blockIdx.x * WPB + wv;        // wave index in the launch
    int rk = 0x7FFFFFFF;
    if constexpr (WPB == 4) rk = kept_rank(a, (int64_t)wblk * ROWS_PER_WAVE + rowi);
    stage_body_table(a, Lmodel, 64 * WPB);
    stage_x0(a, Lx0);
    __syncthreads();
    if constexpr (WPB == 4) {
        if (a.drawn_ahead) {
            if (blockIdx.x == 0 && wv == 1) block0_sample_writes<64>(a, lane);
            kept_rows_wave(a, (int64_t)wblk * ROWS_PER_WAVE + rowi, lane, rk);
        }
    }
    coop_rows<CK, EN, FROW, 0, false, KC>(a, (int64_t)wblk * ROWS_PER_WAVE + rowi, lane, wblk, lds_kin + wrow * KS,
                                          lds_scr + wrow * LDS_SCR, Lmodel, Lx0);
    if constexpr (WPB == 4) {
        if (a.costs_in_launch) launch_costs<CK, EN, KC>(a, wv, lane, Lmodel);
    } else if constexpr (WPB == 1) {
        // past one round (two waves per SIMD, several rounds): the wave's own rows' objective after
        // its loop, while the launch's other waves still run, instead of fr_step_cost_kernel after it
        if (a.costs_in_launch) {
            __builtin_amdgcn_s_waitcnt(0);   // the wave's own record stores, read back by other lanes
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
            for (int i = 0; i < ROWS_PER_WAVE; i++)
                launch_row_cost<CK, EN, KC>(a, (int64_t)blockIdx.x * ROWS_PER_WAVE + i, lane, Lmodel);
        }
    }
}


// The update's launch: four waves of main rows per workgroup (rollouts [0, xbase)) and four more
// waves, one per SIMD beside each main wave, that evaluate the objective in chunks while the rows
// run (cost_work) and make the next update's draws.  In the workgroups with rows left over (the
// extra rows [xbase, count) plus the folded filter() row, xrows of them, four per workgroup) those
// four waves first carry the rows left over through the horizon, a quarter each (relay_stage).
constexpr int XW = 8;
template <int CK, bool EN>
__global__ __launch_bounds__(64 * XW) __attribute__((amdgpu_waves_per_eu(2, 2))) void fr_coop_x_kernel(FrRolloutArgs a)
{
    constexpr int KS = EN ? LDS_KIN_EN : LDS_KIN;
    __shared__ __attribute__((aligned(16))) double lds_kin[5 * ROWS_PER_WAVE * KS];
    __shared__ __attribute__((aligned(16))) double lds_scr[5 * ROWS_PER_WAVE * LDS_SCR];
    __shared__ double Lmodel[LDS_MODEL];
    __shared__ double Lx0[MAX_X];
    __shared__ int Lflag[LF_N];      // records stored (main waves, relay), kept columns copied
    __shared__ int Lq[Q_N];          // the main waves' steps, chunk counters, the relay's stage
    __shared__ double Lst[64 * 3];   // the relay's (q, qd, E) per lane between stages
    __shared__ __attribute__((aligned(16))) double Lcs[5 * ROWS_PER_WAVE * HC_MAX];   // step costs of the groups' rows
    const int wv = (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int rowi = lane >> 4;
    const int member = relay_member(a);   // of the relay rows this workgroup carries (-1: none)
    const bool xr = member >= 0;
    const int64_t lr = wv < 4 ? (int64_t)(blockIdx.x * 4 + wv) * ROWS_PER_WAVE + rowi
                              : a.xbase + (int64_t)((int)blockIdx.x % RELAY_STRIDE) * ROWS_PER_WAVE + rowi;   // (waves < 5)
    const int rk = (wv < 4 || (wv == 4 && xr)) ? kept_rank(a, lr) : 0x7FFFFFFF;
    stage_body_table(a, Lmodel, 64 * XW);
    stage_x0(a, Lx0);
    if (threadIdx.x < LF_N) Lflag[threadIdx.x] = 0;
    if (threadIdx.x < Q_N) Lq[threadIdx.x] = threadIdx.x < Q_NEXT ? -1 : 0;
    const int ng = xr ? 5 : 4;   // row groups of the objective
    if (threadIdx.x == Q_NEXT + 4) {   // the relay group's first chunk here (none: past every chunk)
        int cb, ce;
        group_chunks(a, 4, cb, ce);
        Lq[Q_NEXT + 4] = xr ? cb : 0x7FFF;
    }
    __syncthreads();
    // main wave w's rows use slots 4 w + i, the relay's rows (whichever wave runs them) 16 + i
    const int slot = wv < 4 ? wv * ROWS_PER_WAVE + rowi : 4 * ROWS_PER_WAVE + rowi;
    double *Lk = lds_kin + slot * KS, *Lw = lds_scr + slot * LDS_SCR;
    if (a.drawn_ahead) {
        if (blockIdx.x == 0 && wv == 1) block0_sample_writes<64>(a, lane);   // off the SIMD of the relay's first stage
        if (wv < 4) kept_rows_wave(a, lr, lane, rk);
        else if (wv == 4 && xr) {   // the relay rows' columns of the steps this member runs
            kept_rows_wave(a, lr, lane, rk, relay_member_step(a, member, a.H),
                           member + 1 < a.relay_k ? relay_member_step(a, member + 1, a.H) : 0x7FFFFFFF);
            __hip_atomic_store(Lflag + LF_KEPT_X, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    const bool cil = a.costs_in_launch != 0;
    if (wv < 4) {
        if (cil) {   // the next draws for this wave's rows may now overwrite their previous eps
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(Lflag + LF_KEPT + wv, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_s_setprio(1);   // above the objective's waves, below the relay
        }
        const int wblk = blockIdx.x * 4 + wv;
        coop_rows<CK, EN, false, 0, true>(a, (int64_t)wblk * ROWS_PER_WAVE + rowi, lane, wblk, Lk, Lw, Lmodel, Lx0,
                                          nullptr, 0, 0x7FFFFFFF, Lq + Q_PROG + wv);
        __builtin_amdgcn_s_setprio(0);
        if (cil) {
            signal_records(Lflag + wv);
            cost_work<CK, EN>(a, wv, ng, lane, Lmodel, Lcs, Lflag, Lq);
        }
#ifdef COST_TRACE   // COOP_TRACE builds: slot 3 = the wave's end (after its objective work)
        if (a.trace && lane == 0) a.trace[4 * wblk + 3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
    } else {
        const int s = wv - 4;   // this wave's SIMD
        const bool relay = xr && (s == 0 || a.handover);
        if (relay) relay_stage<CK, EN>(a, s, member, lane, Lk, Lw, Lmodel, Lx0, Lflag, Lq, Lst);
        if (!cil) return;
        // the draws for main wave s's rows (relay stages made theirs before their stage; wave 0's
        // rows of a workgroup with rows left over are left to rank_draw_kernel)
        if (a.ahead_noise && !relay && !(member == 0 && s == 0)) group_draws(a, s, lane, Lflag);
        cost_work<CK, EN>(a, s, ng, lane, Lmodel, Lcs, Lflag, Lq);
    }
}

namespace mppi_eng {

// The device's CU count is the handle's (EnvSwitches::cus, hipDeviceAttributeMultiprocessorCount
// at create): one round of workgroups is one per CU
static int64_t cu_count(const EnvSwitches &env) { return env.cus ? (int64_t)env.cus : 256; }

// Dynamic LDS that lifts a multi-wave workgroup above half of the CU's 160 KiB, so that the
// dispatcher places one workgroup per CU (one wave per SIMD) whatever the kernel's static LDS
// (which the compiler trims per variant): two workgroups on a CU would double up its SIMDs.
template <typename K>
static unsigned one_per_cu_pad(K kernel, int wpb)
{
    if (wpb == 1) return 0;
    hipFuncAttributes at{};
    if (hipFuncGetAttributes(&at, reinterpret_cast<const void *>(kernel)) != hipSuccess) return 0;
    const size_t want = 80 * 1024 + 256;
    return at.sharedSizeBytes >= want ? 0u : (unsigned)(want - at.sharedSizeBytes);
}

template <int CK, bool EN, int WPB, bool FROW, bool KC>
static void launch_k(const FrRolloutArgs &a, unsigned nb, hipStream_t s)
{
    static const unsigned pad = one_per_cu_pad(fr_coop_kernel<CK, EN, WPB, FROW, KC>, WPB);
    hipLaunchKernelGGL((fr_coop_kernel<CK, EN, WPB, FROW, KC>), dim3(nb), dim3(64 * WPB), pad, s, a);
}

template <int CK, bool EN>
static void launch_x(const FrRolloutArgs &a, unsigned nb, hipStream_t s)
{
    static const unsigned pad = one_per_cu_pad(fr_coop_x_kernel<CK, EN>, XW);
    hipLaunchKernelGGL((fr_coop_x_kernel<CK, EN>), dim3(nb), dim3(64 * XW), pad, s, a);
}

template <int WPB, bool FROW, bool KC>
static void launch_one(const FrRolloutArgs &a, unsigned nb, hipStream_t s)
{
    if (a.cost_kind == CK_TRACK_POINT) launch_k<CK_TRACK_POINT, false, WPB, FROW, KC>(a, nb, s);
    else if (a.energy) launch_k<CK_ASSISTED_MANIPULATION, true, WPB, FROW, KC>(a, nb, s);
    else launch_k<CK_ASSISTED_MANIPULATION, false, WPB, FROW, KC>(a, nb, s);
}

bool fr_coop_compact(const FrRolloutArgs &a) { return !a.optimal; }

hipError_t launch_fr_coop(const FrRolloutArgs &a, hipStream_t s)
{
    const unsigned nb = (unsigned)((a.count + ROWS_PER_WAVE - 1) / ROWS_PER_WAVE);
    if (nb == 0) return hipSuccess;
    if (fr_coop_compact(a)) launch_one<1, false, true>(a, nb, s);
    else launch_one<1, false, false>(a, nb, s);   // the standalone filter() row
    return hipGetLastError();
}

hipError_t launch_fr_body_table(const DevModel *model, const DevCost *cost, double *table, hipStream_t s)
{
    hipLaunchKernelGGL(fr_body_table_kernel, dim3(1), dim3(640), 0, s, model, cost, table);
    return hipGetLastError();
}

// The A/B switches (EnvSwitches, the handle's copy): MPPI_COSTS_IN_LAUNCH=0 keeps the separate
// fr_step_cost_kernel; MPPI_HANDOVER=0 leaves the rows left over on wave 4 for the whole horizon,
// beside main wave 0, instead of the relay; MPPI_SPLIT=0 runs rows just past two waves per SIMD as
// one-wave workgroups.
bool fr_coop_costs_in_launch(const EnvSwitches &env) { return !env.costs_in_launch_off; }

// Whether `count` rows run as two fr_coop_x_kernel launches (launch_fr_coop_update): one-wave
// workgroups hold two waves per SIMD, 32 rows per CU and round (8192 on 256 CUs), and a count just
// past that - R = S + 2 at S = 8192, configs[4]'s share per GPU - leaves one wave for a second
// round that runs alone for the whole horizon (1.49 + 1 lone-wave horizons, plus the separate cost
// kernel).  Two launches of one wave per SIMD (each 1.06-1.1 lone-wave horizons with the objective
// beside the loops) take less: the first over one round of full four-wave groups, the second over
// the rest, whose rows left over and the folded filter() row travel through its relay.
bool fr_coop_update_split(int64_t count, const EnvSwitches &env)
{
    constexpr int64_t WG_ROWS = 4 * ROWS_PER_WAVE;
    const int64_t round = cu_count(env) * WG_ROWS;
    if (count <= 2 * round || env.split_off) return false;
    const int64_t rest = count - round, gb = rest / WG_ROWS, xb = rest - gb * WG_ROWS + 1;   // + a folded filter() row
    return gb > 0 && gb <= cu_count(env) && xb <= gb * ROWS_PER_WAVE;
}

// Whether launch_fr_coop_update runs rounds of four-wave groups (the launches that can sample
// their kept rows, a.drawn_ahead) for `count` rows: one round, or the two launches of the split.
bool fr_coop_update_fusable(int64_t count, const EnvSwitches &env)
{
    constexpr int64_t WG_ROWS = 4 * ROWS_PER_WAVE;
    const int64_t groups = count / WG_ROWS, xrows = count - groups * WG_ROWS + 1;   // + a folded filter() row
    return (groups > 0 && groups <= cu_count(env) && xrows <= groups * ROWS_PER_WAVE) || fr_coop_update_split(count, env);
}

bool fr_coop_update_folds(int64_t count, int H, const EnvSwitches &env)
{
    if (env.costs_in_launch_off || H > HC_MAX) return false;
    if (fr_coop_update_split(count, env)) return true;
    constexpr int64_t WG_ROWS = 4 * ROWS_PER_WAVE;
    const int64_t groups = count / WG_ROWS, extra = count - groups * WG_ROWS;
    return extra > 0 && groups > 0 && groups <= cu_count(env) && extra + 1 <= groups * ROWS_PER_WAVE;
}

bool fr_coop_is_update_kernel(const void *f)
{
    return f == (const void *)&fr_coop_x_kernel<CK_ASSISTED_MANIPULATION, false> ||
           f == (const void *)&fr_coop_x_kernel<CK_ASSISTED_MANIPULATION, true> ||
           f == (const void *)&fr_coop_x_kernel<CK_TRACK_POINT, false>;
}

static void launch_x_any(const FrRolloutArgs &a, unsigned nb, hipStream_t s)
{
    if (a.cost_kind == CK_TRACK_POINT) launch_x<CK_TRACK_POINT, false>(a, nb, s);
    else if (a.energy) launch_x<CK_ASSISTED_MANIPULATION, true>(a, nb, s);
    else launch_x<CK_ASSISTED_MANIPULATION, false>(a, nb, s);
}

// The arguments of a launch over rows [r0, r0 + n) of `a`'s shard: the row-indexed buffers start at
// row r0 and the shard at begin + r0, so the kernels' launch-relative row lr is row r0 + lr of the
// update (global rollout begin + r0 + lr: the Philox counter, the rank, the cost slot).
static FrRolloutArgs row_slice(const FrRolloutArgs &a, int64_t r0, int64_t n)
{
    FrRolloutArgs b = a;
    b.begin += r0;
    b.count = n;
    b.noise += r0 * FR_C;   // [H][Rpad][C]: row lr of step k at (k Rpad + lr) C
    b.rec += r0 * a.H * FR_REC;
    b.samp.begin += r0;
    b.samp.count = n;
    b.samp.noise += r0 * FR_C;
    b.samp.prev += r0 * FR_C;
    if (b.ahead_noise) b.ahead_noise += r0 * FR_C;
    return b;
}

// Relay members for a launch of `groups` workgroups with xrows rows left over (a.relay_k): the
// engine's exchange buffer (a.rx), the hand-over, a member workgroup q + RELAY_STRIDE m in the grid for
// every relay group q, at least one chunk and four steps per member; else one workgroup.  Two by
// default: at 4096 x 64 (profiles/r06/relay_k) K = 2 ran 0.1838-0.1848 ms/update against 0.1881-0.1892
// for K = 1, 0.1858-0.1880 for K = 3 and 0.1871-0.1879 for K = 4 (each member's first stage pays
// ~10 us of hand-over and its own setup, so more members stop paying off past two); with gj_rows
// K = 2 0.1757-0.1772, K = 1 0.1789-0.1823, K = 3 0.1776-0.1791 (ab_gjrows.txt).
constexpr int RELAY_K_DEFAULT = 2;
static int relay_members(const FrRolloutArgs &a, int64_t groups, int64_t xrows, const EnvSwitches &env)
{
    if (!a.handover || a.rx == nullptr || xrows <= 0) return 1;
    const int64_t nxb = (xrows + ROWS_PER_WAVE - 1) / ROWS_PER_WAVE;
    const int nch = (a.H + CH - 1) / CH;
    int K = std::min(env.relay_k ? env.relay_k : RELAY_K_DEFAULT, RELAY_K_MAX);
    K = std::min(K, nch);
    if (nxb > RELAY_GROUPS_MAX) return 1;
    for (; K > 1; K--) {
        if (nxb + (int64_t)RELAY_STRIDE * (K - 1) > groups) continue;
        bool ok = true;
        for (int m = 0; m < K && ok; m++) {
            const int k0 = m == 0 ? 0 : (m * nch / K) * CH - 1, k1 = m + 1 == K ? a.H - 1 : ((m + 1) * nch / K) * CH - 1;
            ok = k1 - k0 >= 4;
        }
        if (ok) break;
    }
    return K;
}

// The update's rollouts.  e0 / e1 (may be null): timing events around the rollout launch.
hipError_t launch_fr_coop_update(const FrRolloutArgs &a0, const EnvSwitches &env, hipStream_t s, hipEvent_t e0, hipEvent_t e1, bool *folded,
                                 bool *costs_done, bool *tail_drawn, FrRolloutArgs *final, bool *x_kernel, bool dry,
                                 CoopTail *tail, FrRolloutArgs *final2)
{
    *costs_done = false;
    *tail_drawn = false;
    if (x_kernel) *x_kernel = false;
    if (tail) *tail = CoopTail{};
    constexpr int64_t WG_ROWS = 4 * ROWS_PER_WAVE;
    *folded = false;
    if (fr_coop_update_split(a0.count, env)) {   // two launches: one round of full groups, then the rest
        const int64_t n0 = cu_count(env) * WG_ROWS, rest = a0.count - n0;
        FrRolloutArgs a = a0;
        a.costs_in_launch = !env.costs_in_launch_off && a.H <= HC_MAX ? 1 : 0;
        a.handover = env.handover_off ? 0 : 1;
        if (!a.costs_in_launch || !a.drawn_ahead) a.ahead_noise = nullptr;
        FrRolloutArgs A = row_slice(a, 0, n0), B = row_slice(a, n0, rest);
        A.fcost = nullptr;   // the previous filter() rides with the rows left over
        A.xbase = n0;
        A.xrows = 0;
        const int64_t gb = rest / WG_ROWS, xb = rest - gb * WG_ROWS;
        const bool frow = a0.fcost != nullptr;
        if (!frow) B.fcost = nullptr;
        B.xbase = gb * WG_ROWS;
        B.xrows = xb + (frow ? 1 : 0);
        A.relay_k = 1;
        B.relay_k = relay_members(B, gb, B.xrows, env);
        *folded = frow;
        *costs_done = a.costs_in_launch != 0;
        *tail_drawn = a.ahead_noise != nullptr;
        if (final) *final = A;
        if (final2) *final2 = B;
        if (x_kernel) *x_kernel = true;
        if (tail) *tail = CoopTail{n0, n0 + B.xbase, (int)((B.xrows + 3) / 4), 2};
        if (dry) return hipSuccess;
        if (e0) (void)hipEventRecord(e0, s);
        launch_x_any(A, (unsigned)cu_count(env), s);
        launch_x_any(B, (unsigned)gb, s);
        if (e1) (void)hipEventRecord(e1, s);
        return hipGetLastError();
    }
    const int64_t groups = a0.count / WG_ROWS, extra = a0.count - groups * WG_ROWS;
    // the previous update's filter() rides along when there are extra rows anyway (the fifth wave
    // of the first workgroup has room); alone it would add a wave, so then it stays pending
    const bool frow = a0.fcost != nullptr && extra > 0;
    const int64_t xrows = extra + (frow ? 1 : 0);
    FrRolloutArgs a = a0;
    if (groups == 0 || groups > cu_count(env) || xrows > groups * ROWS_PER_WAVE) {
        if (a.drawn_ahead) return hipErrorInvalidValue;   // the one-wave launch samples nothing
        a.fcost = nullptr;   // more than one round of workgroups: one-wave workgroups throughout
        a.ahead_noise = nullptr;
        a.relay_k = 1;
        a.costs_in_launch = groups > 0 && !env.costs_in_launch_off ? 1 : 0;   // each wave its own rows'
        *costs_done = a.costs_in_launch != 0;
        if (final) *final = a;
        if (dry) return hipSuccess;
        if (e0) (void)hipEventRecord(e0, s);
        const hipError_t e = launch_fr_coop(a, s);
        if (e1) (void)hipEventRecord(e1, s);
        return e;
    }
    if (!frow) a.fcost = nullptr;
    a.xbase = groups * WG_ROWS;
    a.xrows = xrows;
    *folded = frow;
    a.costs_in_launch = !env.costs_in_launch_off && a.H <= HC_MAX ? 1 : 0;   // Lcs holds HC_MAX steps
    a.handover = env.handover_off ? 0 : 1;
    a.relay_k = relay_members(a, groups, xrows, env);
    *costs_done = a.costs_in_launch != 0;
    // tail draws ride in launch_costs of fr_coop_x_kernel only, and need the sampling arguments
    if (xrows == 0 || !a.costs_in_launch || !a.drawn_ahead) a.ahead_noise = nullptr;
    *tail_drawn = a.ahead_noise != nullptr;
    if (final) *final = a;
    if (x_kernel) *x_kernel = xrows != 0;
    if (tail) *tail = CoopTail{0, a.xbase, (int)((xrows + 3) / 4), 1};
    if (dry) return hipSuccess;
    if (e0) (void)hipEventRecord(e0, s);
    if (xrows == 0) launch_one<4, false, true>(a, (unsigned)groups, s);
    else launch_x_any(a, (unsigned)groups, s);
    if (e1) (void)hipEventRecord(e1, s);
    return hipGetLastError();
}

}  // namespace mppi_eng
