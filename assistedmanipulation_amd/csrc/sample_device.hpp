// sample_device.hpp — one piece of Trajectory::sample (mppi.cpp:189-270) on the device: the eps
// column piece of a (step, local rollout), shared by sample_kernel (kernels.hip) and the rollout
// launch's sampling prologue (fr_coop.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"

namespace mppi_sample {

using namespace mppi_eng;

// Device Philox mode: the counter of (global rollout g, step k).  A rollout's draws then do not
// depend on its rank in the previous costs' stable order, so the next update's draws can be made
// before that order and the next state and time exist (draws ahead, engine.cpp); the kept
// rollouts' shifted columns are copied in afterwards.  The injected stream is consumed in the
// reference's draw order (mppi.cpp:242-262), so host-driven parity runs see the reference's noise.
__device__ __forceinline__ int64_t philox_index(int64_t g, int k, int H) { return g * H + k; }

// eps = T z for one draw.  z from the Philox stream keyed by (seed, update, draw).
__device__ __forceinline__ void philox_draw(const SampleParams &P, int64_t draw, const double *T, int C, double *eps)
{
    float z[16];
#pragma unroll
    for (int blk = 0; blk < 4; blk++) {
        if (4 * blk >= C) break;
        mppi_dev::u32x4 ctr{(uint32_t)draw, (uint32_t)((uint64_t)draw >> 32), (uint32_t)P.update_index, (uint32_t)blk};
        mppi_dev::u32x4 r = mppi_dev::philox4x32_10(ctr, (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
        mppi_dev::box_muller(r.x, r.y, z[4 * blk + 0], z[4 * blk + 1]);
        mppi_dev::box_muller(r.z, r.w, z[4 * blk + 2], z[4 * blk + 3]);
    }
    if (P.tdiag) {
        for (int c = 0; c < C; c++) eps[c] = T[c * C + c] * (double)z[c];
    } else {
        for (int i = 0; i < C; i++) {
            double s = 0.0;
            for (int j = 0; j < C; j++) s += T[i * C + j] * (double)z[j];
            eps[i] = s;
        }
    }
}

// The eps column (k) of rollout g as Trajectory::sample leaves it (mppi.cpp:242-269).
// `col` holds the previous contents of the column on entry.
__device__ __forceinline__ void sample_column(const SampleParams &P, int64_t g, int rank, int64_t k, int H, int C,
                                              const double *Uprev, const double *inj, const double *T,
                                              const double *noise, int64_t Rpad, int64_t lr, double *eps)
{
    if (g == 1) {   // m_rollouts[1].noise = -m_optimal_control
        for (int c = 0; c < C; c++) eps[c] = -Uprev[k * C + c];
        return;
    }
    int64_t draw = -1;
    if (rank < P.keep) {
        if (P.shift_by > 0) {
            if (k < P.shifted) {
                for (int c = 0; c < C; c++) eps[c] = noise[((k + P.shift_by) * Rpad + lr) * C + c];
                return;
            }
            draw = (int64_t)rank * (H - P.shifted) + (k - P.shifted);
        } else {
            for (int c = 0; c < C; c++) eps[c] = noise[(k * Rpad + lr) * C + c];
            return;
        }
    } else {
        draw = P.keep_draws + (int64_t)(rank - P.keep) * H + k;
    }
    if (P.injected) {
        for (int c = 0; c < C; c++) eps[c] = inj[draw * C + c];
    } else {
        philox_draw(P, philox_index(g, (int)k, H), T, C, eps);
    }
}

// The cost statistics emptied for the next update's folds: slot i by thread i (< CS_SLOTS), in the
// finish kernel (after weights_gradient_kernel read them, one launch ahead of the folds).  Device-
// scope atomic exchanges, performed where the folds' atomics are (a plain store would sit in this
// XCD's L2 until the kernel's end-of-launch write-back).
__device__ __forceinline__ void reset_cost_stats(CostStats *st, int i)
{
    if (i >= CS_SLOTS) return;
    atomicExch(&st->kmin[16 * i], ~0ull);
    atomicExch(&st->kmax[16 * i], 0ull);
    atomicExch(&st->count[32 * i], 0u);
}

// U*_shifted row k, component c (mppi.cpp:197-207): U* shifted left by shift_by, the last column
// repeated; only meaningful when shift_by > 0 (otherwise U*_shifted keeps its contents)
__device__ __forceinline__ double shifted_u(const SampleArgs &a, int k, int c)
{
    const int64_t sh = a.sp.shift_by, kept = a.sp.shifted;
    return (k < kept) ? a.Uprev[(k + sh) * a.C + c] : a.Uprev[(a.H - 1) * a.C + c];
}

// eps of step k, rollout g (local lr, stable-order rank `rank`, 0 for g < 2), piece blk (DIAG:
// components 4 blk .. 4 blk + 3, zero past C; else all C): rollout 0 is the zero-noise rollout;
// rollout 1 carries -U*; kept rollouts shift the previous update's eps; the rest draw
// (Philox4x32-10 by philox_index, or the injected stream in the reference's draw order).
template <int C, bool DIAG>
__device__ __forceinline__ void sample_eps(const SampleArgs &a, int k, int64_t lr, int64_t g, int rank, int blk,
                                           double *eps)
{
    constexpr int CW = DIAG ? (C < 4 ? C : 4) : C;
    const int c0 = DIAG ? 4 * blk : 0;
    const int cw = DIAG ? ((C - c0) < 4 ? (C - c0) : 4) : C;
    if (g == 0) {
#pragma unroll
        for (int c = 0; c < CW; c++) eps[c] = 0.0;
    } else if (!DIAG) {
        sample_column(a.sp, g, rank, k, a.H, C, a.Uprev, a.inj, a.T, a.prev, a.Rpad, lr, eps);
    } else {
        const SampleParams &P = a.sp;
        int64_t draw = -1;
        const double *src = nullptr;
        double sgn = 1.0;
        if (g == 1) {
            src = a.Uprev + (int64_t)k * C + c0;
            sgn = -1.0;
        } else if (rank < P.keep) {
            if (P.shift_by > 0) {
                if (k < P.shifted) src = a.prev + (((int64_t)k + P.shift_by) * a.Rpad + lr) * C + c0;
                else draw = (int64_t)rank * (a.H - P.shifted) + (k - P.shifted);
            } else {
                src = a.prev + ((int64_t)k * a.Rpad + lr) * C + c0;
            }
        } else {
            draw = P.keep_draws + (int64_t)(rank - P.keep) * a.H + k;
        }
        if (src) {
#pragma unroll
            for (int c = 0; c < CW; c++) eps[c] = (c < cw) ? sgn * src[c] : 0.0;
        } else if (P.injected) {
#pragma unroll
            for (int c = 0; c < CW; c++) eps[c] = (c < cw) ? a.inj[draw * C + c0 + c] : 0.0;
        } else {
            draw = philox_index(g, k, a.H);
            mppi_dev::u32x4 ctr{(uint32_t)draw, (uint32_t)((uint64_t)draw >> 32), (uint32_t)P.update_index, (uint32_t)blk};
            mppi_dev::u32x4 r = mppi_dev::philox4x32_10(ctr, (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
            float z[4];
            mppi_dev::box_muller(r.x, r.y, z[0], z[1]);
            mppi_dev::box_muller(r.z, r.w, z[2], z[3]);
#pragma unroll
            for (int c = 0; c < CW; c++) eps[c] = (c < cw) ? a.tdv[c0 + c] * (double)z[c] : 0.0;
        }
    }
}

// Branch-free form of sample_eps<C, true> for full pieces (C % 4 == 0): where the piece comes
// from.  use_p: sgn * p[0..3] (rollout 0 reads a dummy with sgn 0, rollout 1 -U*, kept rollouts the
// previous eps, injected draws the stream); else a Philox draw `draw`.  Lets a thread issue the
// loads of several pieces before waiting on any (fused_sample_rows).
struct EpsPlan {
    const double *p;
    double sgn;
    int64_t draw;
    bool use_p;
};

template <int C>
__device__ __forceinline__ EpsPlan eps_plan(const SampleArgs &a, int k, int64_t lr, int64_t g, int rank, int blk)
{
    static_assert(C % 4 == 0, "full pieces");
    const SampleParams &P = a.sp;
    const int c0 = 4 * blk;
    EpsPlan e{a.Uprev, 1.0, 0, true};
    if (g == 0) {
        e.sgn = 0.0;
    } else if (g == 1) {
        e.p = a.Uprev + (int64_t)k * C + c0;
        e.sgn = -1.0;
    } else if (rank < P.keep && (P.shift_by <= 0 || k < P.shifted)) {
        e.p = a.prev + (((int64_t)k + (P.shift_by > 0 ? P.shift_by : 0)) * a.Rpad + lr) * C + c0;
    } else {
        if (P.injected) {
            e.draw = rank < P.keep ? (int64_t)rank * (a.H - P.shifted) + (k - P.shifted)
                                   : P.keep_draws + (int64_t)(rank - P.keep) * a.H + k;
            e.p = a.inj + e.draw * C + c0;
        } else {
            e.draw = philox_index(g, k, a.H);
            e.use_p = false;
        }
    }
    return e;
}

// The piece of a plan: v = the four doubles at plan.p (loaded by the caller).
__device__ __forceinline__ void eps_finish(const SampleArgs &a, const EpsPlan &e, int blk, const double *v, double *eps)
{
    if (e.use_p) {
#pragma unroll
        for (int c = 0; c < 4; c++) eps[c] = e.sgn == 0.0 ? 0.0 : e.sgn * v[c];   // rollout 0: +0, as sampled
    } else {
        const SampleParams &P = a.sp;
        mppi_dev::u32x4 ctr{(uint32_t)e.draw, (uint32_t)((uint64_t)e.draw >> 32), (uint32_t)P.update_index, (uint32_t)blk};
        mppi_dev::u32x4 r = mppi_dev::philox4x32_10(ctr, (uint32_t)P.seed, (uint32_t)(P.seed >> 32));
        float z[4];
        mppi_dev::box_muller(r.x, r.y, z[0], z[1]);
        mppi_dev::box_muller(r.z, r.w, z[2], z[3]);
#pragma unroll
        for (int c = 0; c < 4; c++) eps[c] = a.tdv[4 * blk + c] * (double)z[c];
    }
}

// Store one eps piece (sample_eps) into the eps tensor [H][Rpad][C].
template <int C, bool DIAG>
__device__ __forceinline__ void store_eps(const SampleArgs &a, int k, int64_t lr, int blk, const double *eps)
{
    constexpr int CW = DIAG ? (C < 4 ? C : 4) : C;
    const int c0 = DIAG ? 4 * blk : 0;
    const int cw = DIAG ? ((C - c0) < 4 ? (C - c0) : 4) : C;
    double *o = a.noise + ((int64_t)k * a.Rpad + lr) * C + c0;
    if constexpr (CW == 4) {   // a full piece: two 16-byte stores (C = 12: c0 = 0, 4, 8 doubles, 32-B aligned)
        if (cw == 4) {
            reinterpret_cast<double2 *>(o)[0] = double2{eps[0], eps[1]};
            reinterpret_cast<double2 *>(o)[1] = double2{eps[2], eps[3]};
            return;
        }
    }
#pragma unroll
    for (int c = 0; c < CW; c++)
        if (c < cw) o[c] = eps[c];
}

// eps of step k, local rollout lr, piece blk into the eps tensor.
template <int C, bool DIAG>
__device__ __forceinline__ void sample_item(const SampleArgs &a, int k, int64_t lr, int blk)
{
    constexpr int CW = DIAG ? (C < 4 ? C : 4) : C;
    const int64_t g = a.begin + lr;
    double eps[CW];
    sample_eps<C, DIAG>(a, k, lr, g, g >= 2 ? a.rank[g] : 0, blk, eps);
    store_eps<C, DIAG>(a, k, lr, blk, eps);
}

}  // namespace mppi_sample
