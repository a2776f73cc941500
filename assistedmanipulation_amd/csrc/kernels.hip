// kernels.hip — MPPI device kernels for gfx950 (CDNA4, wave64).
//
// One update of mppi::Trajectory (reference src/controller/mppi.cpp:154-187) is the launch
// sequence issued by engine.cpp:
//
//   rank_kernel      stable order of the previous costs            (sample(), mppi.cpp:222-231)
//   sample_kernel    eps of every (step, rollout); U*_shifted <- shift(U*) (sample(), mppi.cpp:189-270)
//   fr_coop_x_kernel (fr_coop.hip) / pm_rollout_kernel
//                    per rollout: eps columns (kept-shift / fresh draw / -U*), fp64 horizon
//                    rollout of the dynamics and the per-step cost, cost[r]
//                                                                  (mppi.cpp:242-342)
//   [RCCL all-reduce of cost[R] when sharded]
//   weights_gradient_kernel  softmin weights and the partial gradient sum_r w_r eps_r over the
//                    local shard, one launch (optimise(), mppi.cpp:344-418)
//   [RCCL all-reduce of the partial gradient when sharded]
//   finish_kernel    U* += step * g, Savitzky-Golay, clamp          (mppi.cpp:421-447)
//   the optimal rollout (folded into the next rollout launch) / pm_rollout_kernel(optimal)
//                    cost of the new U* (filter(), mppi.cpp:450-479)
//   publish_kernel   U* <- U*_shifted, pack the host-visible block   (mppi.cpp:178-182)
//
// Precision: the rollout runs in fp64.  The reference's cost is dominated by 1e10-scale
// barrier terms (controller/cost.hpp:57-62, 88-93) and a 2e11 self-collision constant, so its
// softmin weights are decided by how many horizon steps breach a barrier; fp32 dynamics flip
// those counts within one or two updates (tools/precision_probe.py).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "pm_model.hpp"
#include "sample_device.hpp"

using namespace mppi_eng;
using mppi_dev::smax;
using mppi_dev::smin;

namespace {

// t0 + k dt exactly as the reference's double expression (mppi.cpp:430, 437): window times are
// compared with ==/< (filter.cpp:94-106), so no FMA contraction here.
__device__ __forceinline__ double step_time(double t0, int k, double dt)
{
#pragma clang fp contract(off)
    return t0 + (double)k * dt;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Rank of each sampled rollout (indices 2..R-1) in the stable order of the previous costs.
// NaN sorts last (the reference's comparator is not a strict weak order with NaN: UB).
// Costs become order-preserving 64-bit keys (-0 == +0, NaN above +inf); rank_i counts keys below
// key_i plus equal keys at lower indices.  O(S log S) in two kernels over chunks of 256:
//   rank_chunk_kernel   chunk-local stable rank by all-pairs compares in LDS; writes rank_i
//                       (local) and the chunk's keys in sorted order;
//   rank_merge_kernel   block (a, g) counts, for each key of chunk a, the keys of a group of
//                       RANK_G other chunks below it (chunks after a: lower_bound) or not above
//                       it (chunks before a: upper_bound, equal keys at lower indices), by
//                       binary searches of the sorted chunks staged in LDS; one atomic per key.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t cost_key(double c)
{
    const double z = c + 0.0;   // -0 -> +0
    const uint64_t b = (uint64_t)__double_as_longlong(z);
    const uint64_t k = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    return isnan(c) ? ~0ull : k;
}

constexpr int RANK_T = 256;   // chunk size (one block)
constexpr int RANK_G = 16;    // chunks searched per merge block

__global__ __launch_bounds__(RANK_T) void rank_chunk_kernel(const double *__restrict__ cost, int64_t S, int *__restrict__ rank,
                                                            uint64_t *__restrict__ sorted)
{
    __shared__ uint64_t kj[RANK_T];
    const int t = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * RANK_T + t;
    const uint64_t ki = (i < S) ? cost_key(cost[2 + i]) : ~0ull;
    kj[t] = ki;
    __syncthreads();
    // pads (key ~0 at the chunk's end) sort after every real key, NaN included
    int lr = 0;
#pragma unroll 8
    for (int u = 0; u < RANK_T; u++) {
        const uint64_t k = kj[u];
        lr += (k < ki || (k == ki && u < t)) ? 1 : 0;
    }
    sorted[(int64_t)blockIdx.x * RANK_T + lr] = ki;
    if (i < S) rank[2 + i] = lr;
}

__global__ __launch_bounds__(RANK_T) void rank_merge_kernel(const double *__restrict__ cost, int64_t S, int *__restrict__ rank,
                                                            const uint64_t *__restrict__ sorted)
{
    __shared__ uint64_t sk[RANK_G * RANK_T];
    const int t = threadIdx.x;
    const int a = blockIdx.x;
    const int nch = (int)((S + RANK_T - 1) / RANK_T);
    const int b0 = blockIdx.y * RANK_G;
    const int nb = (nch - b0) < RANK_G ? (nch - b0) : RANK_G;
    {   // all RANK_G loads in flight before the LDS stores
        uint64_t v[RANK_G];
#pragma unroll
        for (int g = 0; g < RANK_G; g++) v[g] = (g < nb) ? sorted[(int64_t)(b0 + g) * RANK_T + t] : ~0ull;
#pragma unroll
        for (int g = 0; g < RANK_G; g++) sk[g * RANK_T + t] = v[g];
    }
    __syncthreads();
    const int64_t i = (int64_t)a * RANK_T + t;
    if (i >= S) return;
    const uint64_t ki = cost_key(cost[2 + i]);
    int pos[RANK_G];
#pragma unroll
    for (int g = 0; g < RANK_G; g++) pos[g] = 0;
    // branch-free binary searches, RANK_G independent chains per thread
#pragma unroll
    for (int step = RANK_T / 2; step > 0; step >>= 1) {
#pragma unroll
        for (int g = 0; g < RANK_G; g++) {
            const bool before = b0 + g < a;   // chunk b precedes a: equal keys count
            const uint64_t k = sk[g * RANK_T + pos[g] + step - 1];
            pos[g] += (k < ki || (before && k == ki)) ? step : 0;
        }
    }
    int cnt = 0;
#pragma unroll
    for (int g = 0; g < RANK_G; g++) {
        const int b = b0 + g;
        // the last position (RANK_T - 1) is never probed: add it when every probe passed
        const uint64_t kl = sk[g * RANK_T + RANK_T - 1];
        const int p = pos[g] + ((pos[g] == RANK_T - 1 && (kl < ki || (b < a && kl == ki))) ? 1 : 0);
        const int64_t nb_b = (S - (int64_t)b * RANK_T) < RANK_T ? (S - (int64_t)b * RANK_T) : RANK_T;   // real keys
        cnt += (g < nb && b != a) ? (p < nb_b ? p : (int)nb_b) : 0;
    }
    if (cnt) atomicAdd(&rank[2 + i], cnt);
}


// Small S (<= RANK_TILED_MAX): all-pairs in tiles, one launch.  Grid (ceil(S/256), ceil(S/256)):
// block (x, y) ranks its 256 rollouts against the 256 of tile y staged in LDS; off the diagonal
// tile the index tie-break is block-uniform, so one compare per pair.  rank[] is zeroed by the
// finish kernel that precedes this launch on the engine stream.
__device__ __forceinline__ void rank_tile(const double *__restrict__ cost, int64_t S, int *__restrict__ rank, unsigned bx,
                                          unsigned by, uint64_t *kj, unsigned js = 0, unsigned ns = 1);

__global__ __launch_bounds__(RANK_T) void rank_tiled_kernel(const double *__restrict__ cost, int64_t S, int *__restrict__ rank)
{
    __shared__ uint64_t kj[RANK_T];
    rank_tile(cost, S, rank, blockIdx.x, blockIdx.y, kj);
}

// (js, ns): the block compares against columns [js W, (js + 1) W) of tile by only, W = RANK_T / ns
// (ns blocks per tile: a chain of W compares per thread instead of RANK_T)
__device__ __forceinline__ void rank_tile(const double *__restrict__ cost, int64_t S, int *__restrict__ rank, unsigned bx,
                                          unsigned by, uint64_t *kj, unsigned js, unsigned ns)
{
    const int W = RANK_T / (int)ns;
    const int64_t i = (int64_t)bx * RANK_T + threadIdx.x;
    const int64_t j0 = (int64_t)by * RANK_T + (int64_t)js * W;
    const int64_t jl = j0 + threadIdx.x;
    if ((int)threadIdx.x < W) kj[threadIdx.x] = (jl < S) ? cost_key(cost[2 + jl]) : ~0ull;
    __syncthreads();
    if (i >= S) return;
    const uint64_t ki = cost_key(cost[2 + i]);
    const int jn = (int)((S - j0) < W ? (S - j0) : W);
    int cnt = 0;
    if (by < bx) {          // every j < i: equal keys count
#pragma unroll 8
        for (int t = 0; t < jn; t++) cnt += (kj[t] <= ki) ? 1 : 0;
    } else if (by > bx) {   // every j > i
#pragma unroll 8
        for (int t = 0; t < jn; t++) cnt += (kj[t] < ki) ? 1 : 0;
    } else {
        const int il = (int)threadIdx.x - (int)js * W;   // this row's column in the block's range
        for (int t = 0; t < jn; t++) cnt += (kj[t] < ki || (kj[t] == ki && t < il)) ? 1 : 0;
    }
    if (cnt) atomicAdd(&rank[2 + i], cnt);
}

// sample(): eps column k of local rollout lr (mppi.cpp:242-269).  Rollout 0 is the zero-noise
// rollout; rollout 1 carries -U*; kept rollouts shift the previous update's eps; the rest draw.
// Diagonal noise transform: one thread per (step, rollout, Philox block of 4 components), so
// consecutive threads write consecutive 32-byte pieces of step k's [Rpad][C] slab.  Full
// transform: one thread per (step, rollout) (eps = T z needs all C normals of the draw).
// grid (ceil(count * NB / 256), H).  Block (0, k) also writes U*_shifted row k (mppi.cpp:197-207).
template <int C, bool DIAG>
__global__ __launch_bounds__(256) void sample_kernel(SampleArgs a)
{
    constexpr int NB = DIAG ? (C + 3) / 4 : 1;   // thread pieces per (step, rollout)
    const int k = blockIdx.y;
    if (blockIdx.x == 0 && k == 0 && (int)threadIdx.x < a.X) a.x0_out[threadIdx.x] = a.x0v[threadIdx.x];
    if (blockIdx.x == 0 && a.sp.shift_by > 0 && (int)threadIdx.x < C) {
        const int c = threadIdx.x;
        a.Us[k * C + c] = mppi_sample::shifted_u(a, k, c);
    }
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t lr = tid / NB;
    if (lr >= a.count) return;
    mppi_sample::sample_item<C, DIAG>(a, k, lr, (int)(tid - lr * NB));
}

// The next update's draws, ahead (engine.cpp): every local rollout's eps for every step as if
// nothing were kept.  Rollout 0 zero, rollout 1 = -U* (the U* just published), the rest Philox by
// (rollout, step) (sample_device.hpp philox_index).  The update's rollout launch copies the kept
// rollouts' shifted columns over these once the shift is known (fr_coop.hip kept_columns).
template <int C>
__device__ __forceinline__ void draw_ahead_block(const SampleArgs &a, unsigned bx, int k, int sub_nxb, int64_t sub_xbase,
                                                 int64_t sub_row0)
{
    static_assert(C % 4 == 0, "full pieces");
    constexpr int NB = C / 4;
    const int64_t tid = (int64_t)bx * 256 + threadIdx.x;
    int64_t lr = tid / NB;
    const int blk = (int)(tid - lr * NB);
    if (sub_nxb > 0) {   // only the rows the rollout launch's tail left (fr_coop.hip tail_draws)
        const int64_t nm = 4 * (int64_t)sub_nxb, nx = a.count - sub_xbase;
        // and, when those rows are not the first launch's, rollouts 0 and 1 (-U*), which no
        // launch draws (their first wave's rows: tail_draws skips g < 2)
        const int64_t lead01 = (sub_row0 > 0 && a.begin < 2) ? 2 - a.begin : 0;
        if (lr < nm) lr = sub_row0 + 16 * (lr / 4) + (lr % 4);
        else if (lr < nm + nx) lr = sub_xbase + (lr - nm);
        else lr = lr < nm + nx + lead01 ? lr - nm - nx : a.count;   // past the rows: none
    }
    if (lr >= a.count) return;
    const int64_t g = a.begin + lr;
    mppi_sample::EpsPlan e{a.Uprev, 0.0, 0, true};   // rollout 0: zeros
    if (g == 1) {
        e.p = a.Uprev + (int64_t)k * C + 4 * blk;
        e.sgn = -1.0;
    } else if (g >= 2) {
        e.draw = mppi_sample::philox_index(g, k, a.H);
        e.use_p = false;
    }
    double v[4] = {0.0, 0.0, 0.0, 0.0}, eps[4];
    if (e.use_p) {
        const double2 *p2 = reinterpret_cast<const double2 *>(e.p);
        const double2 lo = p2[0], hi = p2[1];
        v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
    }
    mppi_sample::eps_finish(a, e, blk, v, eps);
    mppi_sample::store_eps<C, true>(a, k, lr, blk, eps);
}

constexpr unsigned RANK_JS = 4;   // blocks per rank tile: its 256 columns split four ways (r02i)
// The draws ahead and the stable rank of this update's costs in one launch (neither reads the
// other's output): blocks [0, nr^2) rank tiles, the rest draw (grid nx x H flattened)
template <int C>
__global__ __launch_bounds__(256) void rank_draw_kernel(const double *__restrict__ cost, int64_t S, int *__restrict__ rank,
                                                        unsigned nr, SampleArgs a, unsigned nx, int sub_nxb, int64_t sub_xbase,
                                                        int64_t sub_row0)
{
    __shared__ uint64_t kj[RANK_T];
    static_assert(RANK_T == 256, "one block size");
    const unsigned b = blockIdx.x;
    const unsigned nrb = nr * nr * RANK_JS;
    if (b < nrb) rank_tile(cost, S, rank, b % nr, (b / nr) % nr, kj, b / (nr * nr), RANK_JS);
    else {
        const unsigned d = b - nrb;
        draw_ahead_block<C>(a, d % nx, (int)(d / nx), sub_nxb, sub_xbase, sub_row0);
    }
}

hipError_t mppi_eng::launch_draw_ahead(const SampleArgs &a, const double *cost, int64_t S, int *rank, uint64_t *sorted,
                                       hipStream_t s, int sub_nxb, int64_t sub_xbase, int64_t sub_row0, RankDrawLaunch *out,
                                       bool dry)
{
    if (a.C != FR_C || a.count <= 0) return hipErrorInvalidValue;
    if (sub_nxb > 0 && (sub_row0 < 0 || sub_row0 + 16 * (int64_t)sub_nxb > sub_xbase || sub_xbase > a.count))
        return hipErrorInvalidValue;
    constexpr int NB = FR_C / 4;
    const int64_t lead01 = (sub_row0 > 0 && a.begin < 2) ? 2 - a.begin : 0;   // rollouts 0 and 1 (draw_ahead_block)
    const int64_t rows = sub_nxb > 0 ? 4 * (int64_t)sub_nxb + (a.count - sub_xbase) + lead01 : a.count;
    const unsigned nx = (unsigned)((rows * NB + 255) / 256);
    unsigned nr = (unsigned)((S + RANK_T - 1) / RANK_T);
    if (S > RANK_TILED_MAX) {   // O(S log S) rank in its own launches, then the draws alone
        // (dry: the hipGraph replay, whose captured rank launches keep their arguments)
        if (!dry) {
            const hipError_t e = launch_rank(cost, S, rank, sorted, s);
            if (e != hipSuccess) return e;
        }
        nr = 0;
    }
    const unsigned grid = nr * nr * RANK_JS + nx * (unsigned)a.H;
    if (out) *out = RankDrawLaunch{cost, S, rank, nr, nx, a, sub_nxb, sub_xbase, sub_row0, grid};
    if (dry) return hipSuccess;
    hipLaunchKernelGGL((rank_draw_kernel<FR_C>), dim3(grid), dim3(256), 0, s, cost, S, rank, nr, a, nx, sub_nxb, sub_xbase,
                       sub_row0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Point-mass rollouts (config 2).  State (p, v), control = force.
// ---------------------------------------------------------------------------------------------
// One lane per rollout: the horizon is a chain of dependent steps whose loads (the rollout's eps,
// U*_shifted and the step's discount) used to be issued inside it, one memory latency per step
// (19.6 us for 32 steps at 1024 x 32).  The loads now run PM_PF steps ahead: the next block's are
// issued before the current block's arithmetic (the same operations in the same order).
constexpr int PM_PF = 16;
struct PmBlock {
    double e[PM_PF][3], u[PM_PF][3], gm[PM_PF];
};
__device__ __forceinline__ void pm_load(const PmRolloutArgs &a, int64_t lr, int k0, PmBlock &b)
{
#pragma unroll
    for (int j = 0; j < PM_PF; j++) {
        const int k = k0 + j < a.H ? k0 + j : a.H - 1;   // past the horizon: loaded, unused
#pragma unroll
        for (int c = 0; c < 3; c++) {
            b.e[j][c] = a.optimal ? 0.0 : a.noise[((int64_t)k * a.Rpad + lr) * 3 + c];
            b.u[j][c] = a.Ushift[k * 3 + c];
        }
        b.gm[j] = a.steps[k].gamma_k;
    }
}
__device__ __forceinline__ void pm_steps(const PmRolloutArgs &a, const DevPointMass &P, int k0, const PmBlock &b, double *x,
                                         double &J, bool &alive)
{
#pragma unroll
    for (int j = 0; j < PM_PF; j++) {
        if (k0 + j >= a.H || !alive) return;
        double u[3], dv[3], cu;
#pragma unroll
        for (int c = 0; c < 3; c++) u[c] = b.u[j][c] + b.e[j][c];
        pm_control_step(P, u, a.dt, dv, cu);   // pm_model.hpp: the fused launch's operations
        double Jn = J;
        const double sc = pm_state_step(P, x, dv, cu, b.gm[j], a.dt, Jn);
        if (!a.optimal && isnan(sc)) {
            J = NAN;
            alive = false;
            return;
        }
        J = Jn;
    }
}
__global__ __launch_bounds__(256) void pm_rollout_kernel(PmRolloutArgs a)
{
    const int64_t lr = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lr >= a.count) return;
    if (a.optimal && (a.status->all_nan || a.status->sg_error)) return;
    const int64_t g = a.optimal ? -1 : a.begin + lr;
    const DevPointMass &P = *a.pm;
    double x[6];
    for (int i = 0; i < 6; i++) x[i] = a.x0[i];
    double J = 0.0;
    bool alive = true;
    PmBlock b0, b1;   // ping-pong: one block's loads in flight while the other's steps run
    pm_load(a, lr, 0, b0);
    for (int k0 = 0; k0 < a.H; k0 += 2 * PM_PF) {
        if (k0 + PM_PF < a.H) pm_load(a, lr, k0 + PM_PF, b1);
        pm_steps(a, P, k0, b0, x, J, alive);
        if (k0 + PM_PF >= a.H) break;
        if (k0 + 2 * PM_PF < a.H) pm_load(a, lr, k0 + 2 * PM_PF, b0);
        pm_steps(a, P, k0 + PM_PF, b1, x, J, alive);
    }
    if (a.optimal) *a.cost_out = J;
    else a.cost_out[g] = J;
}

// ---------------------------------------------------------------------------------------------
// optimise(): min / max over non-NaN costs, status, softmin weights (mppi.cpp:344-408).
// One workgroup of 1024 threads.
// ---------------------------------------------------------------------------------------------
// Block-wide reductions for one 1024-thread workgroup: wave butterflies, then 16 wave partials.
__device__ __forceinline__ double wave_min(double v) { return mppi_dev::wave_min_dpp(v); }
__device__ __forceinline__ double wave_max(double v) { return mppi_dev::wave_max_dpp(v); }
__device__ __forceinline__ double wave_sum(double v) { return mppi_dev::wave_sum_dpp(v); }

// optimise() and the partial gradient in one launch (mppi.cpp:344-418), grid (H, GRAD_SPLIT).
// Block (k, s) sums e_r eps_r (e_r the unnormalised softmin weight) over a contiguous eighth of the
// local rollouts of step k, one rollout's C contiguous components per thread, then its 256 partials
// in a fixed tree into gsplit[s][k] (deterministic, no atomics); the finish kernel adds the
// GRAD_SPLIT partials in a fixed order and divides by the normaliser total = sum_r e_r:
// (sum_r e_r eps_r) / total for the reference's sum_r (e_r / total) eps_r, a rounding difference.
// e_r needs min / max / count of the costs: every block computes them itself from the costs (out of
// L2) instead of waiting for another block, in the order of one 1024-thread block - each real wave
// carries four of its sixteen waves lane for lane, so the butterflies pair the same values and
// every block holds the same bits.  The normaliser is not needed here: blocks (0, s) write e_r of
// slice s of all R rollouts to wexp and its sum to Status::tsplit[s] (the finish kernel adds them,
// the host divides for get_weights), so no block evaluates all R exponentials; unsharded, slice s
// is block (0, s)'s own rollout range, so its gradient loop makes those e_r (same order, same
// bits) and no second pass runs.  The block's eps and cost loads are issued first, together, and
// land during the reductions.  Block (0, 0) writes the status words.
constexpr int WV = 16;       // waves of the 1024-thread reduction order
constexpr int WU = 2;        // costs per (virtual) thread and pass (min / max / count are exact in any order)
constexpr int NV = WV / 4;   // virtual waves per real wave
constexpr int GR = 3;     // rollouts per thread whose eps is loaded up front (R = 4098: 513 per block)

// Large R (R > SM_LARGE_R, configs 4 / 5: every rank weighs all R global costs): recomputing
// min / max / normaliser over all R in each of the H x GRAD_SPLIT blocks costs O(H R) exps, so
// the reductions run once, in two small launches over SM_NB contiguous chunks:
//   softmin_minmax_kernel   chunk b's min / max / count of the non-NaN costs -> wpart[0..3 NB)
//   softmin_exp_kernel      every block folds the NB partials in one fixed order (same bits in
//                           every block), then writes e_r = exp(-lambda (c_r - min) / (max - min))
//                           of its chunk to wexp and the chunk's sum to wpart[3 NB + b]
// and weights_gradient_kernel<C, true> folds the NB sums the same way for the normaliser and
// reads e_r instead of recomputing it.
constexpr int SM_NB = 64;
constexpr int64_t SM_LARGE_R = 16384;

__device__ __forceinline__ void sm_chunk(int64_t R, int b, int64_t &r0, int64_t &r1)
{
    const int64_t cs = (R + SM_NB - 1) / SM_NB;
    r0 = (int64_t)b * cs;
    r1 = (r0 + cs < R) ? r0 + cs : R;
}

// the NB chunk partials folded by the first wave (lane b holds chunk b): min, max, count [, sum]
__device__ __forceinline__ void sm_fold(const double *wpart, int l, bool with_sum, double &mn, double &mx, double &cn,
                                        double &sm)
{
    static_assert(SM_NB == 64, "one partial per lane");
    mn = wave_min(wpart[l]);
    mx = wave_max(wpart[SM_NB + l]);
    cn = wave_sum(wpart[2 * SM_NB + l]);
    sm = with_sum ? wave_sum(wpart[3 * SM_NB + l]) : 0.0;
}

__global__ __launch_bounds__(256) void softmin_minmax_kernel(WGradArgs a)
{
    __shared__ double smn[4], smx[4], scn[4];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    int64_t r0, r1;
    sm_chunk(a.R, blockIdx.x, r0, r1);
    double mn = INFINITY, mx = -INFINITY, cn = 0.0;
    for (int64_t r = r0 + t; r < r1; r += 256) {
        const double c = a.cost[r];
        const bool ok = !isnan(c);
        cn += ok ? 1.0 : 0.0;
        mn = (ok && c < mn) ? c : mn;
        mx = (ok && c > mx) ? c : mx;
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    cn = wave_sum(cn);
    if (l == 0) { smn[w] = mn; smx[w] = mx; scn[w] = cn; }
    __syncthreads();
    if (t == 0) {
        a.wpart[blockIdx.x] = smin(smin(smn[0], smn[1]), smin(smn[2], smn[3]));
        a.wpart[SM_NB + blockIdx.x] = smax(smax(smx[0], smx[1]), smax(smx[2], smx[3]));
        a.wpart[2 * SM_NB + blockIdx.x] = (scn[0] + scn[1]) + (scn[2] + scn[3]);
    }
}

__global__ __launch_bounds__(256) void softmin_exp_kernel(WGradArgs a)
{
    __shared__ double sfold[3], ssum[4];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    if (w == 0) {
        double mn, mx, cn, sm;
        sm_fold(a.wpart, l, false, mn, mx, cn, sm);
        if (l == 0) { sfold[0] = mn; sfold[1] = mx; sfold[2] = cn; }
    }
    __syncthreads();
    const double minimum = sfold[0], maximum = sfold[1], valid = sfold[2];
    if (valid <= 1.0 || maximum - minimum < 1e-6) return;   // weights_gradient_kernel reports it
    const double difference = maximum - minimum;
    int64_t r0, r1;
    sm_chunk(a.R, blockIdx.x, r0, r1);
    double acc = 0.0;
    for (int64_t r = r0 + t; r < r1; r += 256) {
        const double c = a.cost[r];
        const double e = isnan(c) ? 0.0 : exp(-a.cost_scale * (c - minimum) / difference);
        a.wexp[r] = e;
        acc += e;
    }
    acc = wave_sum(acc);
    if (l == 0) ssum[w] = acc;
    __syncthreads();
    if (t == 0) a.wpart[3 * SM_NB + blockIdx.x] = (ssum[0] + ssum[1]) + (ssum[2] + ssum[3]);
}

// C = FR_C (96-byte eps rows): a block takes two steps (k, k + 1) of split s, so the cost
// statistics' fold and the window's exponentials - the same for every step - are formed once per
// two steps, and the grid is (H / 2) x GRAD_SPLIT = 256 workgroups, one per CU.  The eps are read
// contiguously, eight rollouts (768 B) per wave load on lanes 0..47, lane l always holding
// component pair l % 6 of rollout l / 6 of the octet: a load touches 6 cache lines, where one
// rollout per lane touched 48 for 1 KB.  The loads go through a buffer descriptor per step over the
// block's rows (32-bit offsets, the step's stride in the scalar offset; rows past the block read 0
// from the range check).  The window's e_r go through LDS (rollout 8 o + l / 6 for octet o), and the
// lanes' pair partials are added per component at the end.
constexpr int WG_OCT = 17;              // octet loads per lane, step and window (4 waves x 8 rollouts)
constexpr int WG_WIN = 32 * WG_OCT;     // rollouts per window (544: R = 4098 is 513 per split, one window)
constexpr int WG_KPB = 2;               // steps per workgroup (C = FR_C)
static_assert(WG_WIN <= 256 * GR, "a window's costs are loaded by the GR cost loads");

template <int C, bool LARGE>
__global__ __launch_bounds__(256) void weights_gradient_kernel(WGradArgs a)
{
    constexpr int CP = C;
    constexpr bool OCT = C == FR_C;
    constexpr int KPB = OCT ? WG_KPB : 1;
    typedef double d2v __attribute__((ext_vector_type(2)));
    __shared__ double red[4 * CP];
    __shared__ double smn[WV], smx[WV], ssum[WV];
    __shared__ double es[OCT ? 256 * GR : 1];            // e_r of the window (OCT)
    __shared__ double ored[OCT ? KPB * 4 * 48 * 2 : 1];  // lane pair partials, [step][wave][lane][2] (OCT)
    const int t = threadIdx.x, rw = t >> 6, l = t & 63;
    const int64_t R = a.R;
    const int kb = blockIdx.x * KPB, s = blockIdx.y, ns = gridDim.y;
    const bool k0 = blockIdx.x == 0;   // the block holding step 0
    const int64_t chunk = (a.count + ns - 1) / ns;
    const int64_t r0 = (int64_t)s * chunk, r1 = (r0 + chunk < a.count) ? r0 + chunk : a.count;
    // One memory trip, in this order: the cost statistics (unsharded), the costs (LARGE: e_r), then
    // the eps rows.  Vector memory completes in issue order, so the exponentials - which need only
    // the costs and min / max - are formed while the eps loads are still in flight.
    const bool stats = !LARGE && a.stats != nullptr;
    unsigned long long skn = ~0ull, skx = 0;
    unsigned int scn = 0;
    if (stats) {
        skn = a.stats->kmin[16 * l];
        skx = a.stats->kmax[16 * l];
        scn = a.stats->count[32 * l];
    }
    double cpre[GR];    // the costs of rollouts wb + t + 256 m of the window (LARGE: e_r)
    double ne[OCT ? 1 : GR][OCT ? 1 : CP];   // C != FR_C: their eps
    d2v ov[OCT ? KPB : 1][OCT ? WG_OCT : 1]; // OCT: the window's octet loads per step
    const int pl = l % 6, rl = l / 6;        // OCT: this lane's pair and rollout within an octet
    const bool al = l < 48;
    // OCT: the steps' descriptors over rows [r0, r1) (built from launch-uniform values only)
    __amdgpu_buffer_rsrc_t rs[OCT ? KPB : 1];
    if constexpr (OCT) {
#pragma unroll
        for (int j = 0; j < KPB; j++) {
            const int kk = min(kb + j, a.H - 1);
            rs[j] = __builtin_amdgcn_make_buffer_rsrc((void *)(a.noise + ((int64_t)kk * a.Rpad + r0) * C), (short)0,
                                                      (int)((r1 - r0) * C * 8), 0x00020000);
        }
    }
    auto load_window = [&](int64_t wb) {
#pragma unroll
        for (int m = 0; m < GR; m++) {
            const int64_t r = wb + t + 256 * m;
            const int64_t gi = a.begin + (r < r1 ? r : 0);
            if constexpr (LARGE) cpre[m] = a.wexp[gi];
            else cpre[m] = a.cost[gi];
        }
        if constexpr (OCT) {
            const int noct = (int)((min(r1 - wb, (int64_t)WG_WIN) + 7) / 8);   // octets in the window
            // lanes 48..63 and rows past r1 read 0 (past the descriptor's range)
            const int voff = al ? (int)((wb - r0 + 8 * rw + rl) * (C * 8) + 16 * pl) : 0x7FFFFFF0;
#pragma unroll
            for (int j = 0; j < KPB; j++)
#pragma unroll
                for (int u = 0; u < WG_OCT; u++)
                    if (rw + 4 * u < noct)   // wave-uniform
                        ov[j][u] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs[j], voff, u * 32 * C * 8, 0));
        } else {
#pragma unroll
            for (int m = 0; m < GR; m++) {
                const int64_t r = wb + t + 256 * m;
                const double *n = a.noise + ((int64_t)kb * a.Rpad + (r < r1 ? r : 0)) * C;
#pragma unroll
                for (int c = 0; c < CP; c++) ne[m][c] = n[c];
            }
        }
    };
    load_window(r0);
    // unsharded, the normaliser slice of the step-0 block (0, s) is its own rollout range [r0, r1):
    // its e_r come from the gradient loop below, in the same per-thread order as the slice pass
    const bool own_slice = !LARGE && k0 && a.begin == 0 && a.count == R;
    double minimum, maximum, valid, total;
    if constexpr (LARGE) {
        if (rw == 0) {
            double mn, mx, cn, sm;
            sm_fold(a.wpart, l, true, mn, mx, cn, sm);
            if (l == 0) { smn[0] = mn; smx[0] = mx; ssum[0] = cn; ssum[1] = sm; }
        }
        __syncthreads();
        minimum = smn[0];
        maximum = smx[0];
        valid = ssum[0];
        total = ssum[1];
    } else if (stats) {   // from the objective's atomics (exact: the same values as the pass)
        static_assert(CS_SLOTS == 64, "one slot per lane");
        // the slots' keys decoded (order-preserving: the min / max of the values are the values of
        // the min / max keys), empty slots as +inf / -inf, folded as doubles
        const double vn = skn == ~0ull ? (double)INFINITY : mppi_dev::cost_from_key(skn);
        const double vx = skx == 0ull ? -(double)INFINITY : mppi_dev::cost_from_key(skx);
        const unsigned int n = (unsigned int)mppi_dev::wave_sum_dpp((double)scn);
        minimum = n ? mppi_dev::wave_min_dpp(vn) : (double)INFINITY;
        maximum = n ? mppi_dev::wave_max_dpp(vx) : -(double)INFINITY;
        valid = (double)n;
        total = 0.0;
    } else {
    // min / max / count over the non-NaN costs
    double mn[NV], mx[NV], cn[NV];
#pragma unroll
    for (int v = 0; v < NV; v++) {
        mn[v] = INFINITY;
        mx[v] = -INFINITY;
        cn[v] = 0.0;
    }
    for (int64_t base = 0; base < R; base += WV * 64 * WU) {
        double cv[WU][NV];
#pragma unroll
        for (int u = 0; u < WU; u++)
#pragma unroll
            for (int v = 0; v < NV; v++) {
                const int64_t i = base + (int64_t)u * (WV * 64) + (NV * rw + v) * 64 + l;
                cv[u][v] = (i < R) ? a.cost[i] : (double)NAN;
            }
#pragma unroll
        for (int u = 0; u < WU; u++)
#pragma unroll
            for (int v = 0; v < NV; v++) {
                const double c = cv[u][v];
                const bool ok = !isnan(c);
                cn[v] += ok ? 1.0 : 0.0;
                mn[v] = (ok && c < mn[v]) ? c : mn[v];
                mx[v] = (ok && c > mx[v]) ? c : mx[v];
            }
    }
#pragma unroll
    for (int v = 0; v < NV; v++) {
        const double v0 = wave_min(mn[v]), v1 = wave_max(mx[v]), v2 = wave_sum(cn[v]);
        if (l == 0) {
            smn[NV * rw + v] = v0;
            smx[NV * rw + v] = v1;
            ssum[NV * rw + v] = v2;
        }
    }
    __syncthreads();
    minimum = smn[0];
    maximum = smx[0];
    valid = ssum[0];
#pragma unroll
    for (int i = 1; i < WV; i++) {
        minimum = smin(minimum, smn[i]);
        maximum = smax(maximum, smx[i]);
        valid += ssum[i];
    }

    __syncthreads();
    total = 0.0;
    }
    const bool lead = k0 && s == 0 && t == 0;
    Status *st = a.status;
    if (valid <= 1.0) {   // minmax_element over <= 1 element: it1 == it2 -> throw
        if (lead) { st->all_nan = 1; st->early = 1; st->minimum = minimum; st->maximum = maximum; }
        return;
    }
    const double difference = maximum - minimum;
    if (difference < 1e-6) {   // early return, weights/gradient stale (mppi.cpp:373-375)
        if (lead) { st->all_nan = 0; st->early = 1; st->minimum = minimum; st->maximum = maximum; }
        return;
    }
    auto expw = [&](double c) { return isnan(c) ? 0.0 : exp(-a.cost_scale * (c - minimum) / difference); };
    if constexpr (LARGE) {   // the normaliser is known: one partial carries it
        if (k0 && t < GRAD_SPLIT) st->tsplit[t] = t == 0 ? total : 0.0;
    } else if (k0 && !own_slice) {   // slice s of [0, R): e_r and its sum
        const int64_t wc = (R + ns - 1) / ns, w0 = (int64_t)s * wc, w1 = (w0 + wc < R) ? w0 + wc : R;
        double part = 0.0;
        for (int64_t i = w0 + t; i < w1; i += 256) {
            const double e = expw(a.cost[i]);
            a.wexp[i] = e;
            part += e;
        }
        part = wave_sum(part);
        __syncthreads();   // smn / smx / ssum reads above are done
        if (l == 0) ssum[rw] = part;
        __syncthreads();
        if (t == 0) st->tsplit[s] = (ssum[0] + ssum[1]) + (ssum[2] + ssum[3]);
    }
    if (lead) { st->all_nan = 0; st->early = 0; st->minimum = minimum; st->maximum = maximum; }
    double acc[CP];      // C != FR_C: this thread's rollouts' sum
#pragma unroll
    for (int c = 0; c < CP; c++) acc[c] = 0.0;
    d2v oacc[OCT ? KPB : 1];   // OCT: this lane's pair, per step
#pragma unroll
    for (int j = 0; j < (OCT ? KPB : 1); j++) oacc[j] = d2v{0.0, 0.0};
    double part = 0.0;   // own_slice: this thread's share of the normaliser slice
    for (int64_t wb = r0; wb < r1;) {
        // the window's exponentials (their loads landed with the eps still in flight); OCT windows
        // are WG_WIN rollouts, the GR cost loads may reach past one
        const int64_t we = OCT ? min(r1, wb + WG_WIN) : r1;
        double wr[GR];
#pragma unroll
        for (int m = 0; m < GR; m++) {
            const int64_t r = wb + t + 256 * m;
            if constexpr (LARGE) wr[m] = cpre[m];
            else wr[m] = expw(cpre[m]);
            wr[m] = r < we ? wr[m] : 0.0;
            if (own_slice && r < we) {
                a.wexp[r] = wr[m];
                part += wr[m];
            }
        }
        if constexpr (OCT) {
#pragma unroll
            for (int m = 0; m < GR; m++) es[t + 256 * m] = wr[m];
            __syncthreads();
            const int noct = (int)((min(r1 - wb, (int64_t)WG_WIN) + 7) / 8);
#pragma unroll
            for (int u = 0; u < WG_OCT; u++) {
                const int o = rw + 4 * u;
                if (o < noct) {
                    const double w = es[8 * o + rl];   // zero past r1 (wr above); lanes >= 48 loaded 0
#pragma unroll
                    for (int j = 0; j < KPB; j++) oacc[j] += w * ov[j][u];
                }
            }
        } else {
#pragma unroll
            for (int m = 0; m < GR; m++) {
                const int64_t r = wb + t + 256 * m;
                if (r < r1) {
#pragma unroll
                    for (int c = 0; c < CP; c++) acc[c] += wr[m] * ne[m][c];
                }
            }
        }
        wb += OCT ? WG_WIN : 256 * GR;
        if (wb >= r1) break;
        if constexpr (OCT) __syncthreads();   // es is rewritten by the next window
        load_window(wb);   // ranges past one window (R > 8 x 544): one more memory trip per window
    }
    if (own_slice) {   // as the slice pass: butterflies, then the four wave sums in order
        part = wave_sum(part);
        if (l == 0) ssum[rw] = part;
    }
    if constexpr (OCT) {
        // component c = 2 p + i of step kb + j: the 32 lane partials of pair p (lanes p + 6 q of the
        // four waves), in wave order
        if (al)
#pragma unroll
            for (int j = 0; j < KPB; j++) {
                ored[((j * 4 + rw) * 48 + l) * 2] = oacc[j][0];
                ored[((j * 4 + rw) * 48 + l) * 2 + 1] = oacc[j][1];
            }
        __syncthreads();
        if (t < KPB * CP) {
            const int j = t / CP, c = t % CP, p = c >> 1, i = c & 1;
            double g = 0.0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                double gw = 0.0;
#pragma unroll
                for (int q = 0; q < 8; q++) gw += ored[((j * 4 + w) * 48 + p + 6 * q) * 2 + i];
                g += gw;
            }
            if (kb + j < a.H) a.gsplit[((int64_t)s * a.H + kb + j) * C + c] = g;
        }
    } else {
        // the block's 256 partials: butterflies within each wave, then the four wave sums in order
#pragma unroll
        for (int c = 0; c < CP; c++) acc[c] = wave_sum(acc[c]);
        if (l == 0)
#pragma unroll
            for (int c = 0; c < CP; c++) red[rw * CP + c] = acc[c];
        __syncthreads();
        if (t < CP)
            a.gsplit[((int64_t)s * a.H + kb) * C + t] = (red[t] + red[CP + t]) + (red[2 * CP + t] + red[3 * CP + t]);
    }
    if (own_slice && t == 0) st->tsplit[s] = (ssum[0] + ssum[1]) + (ssum[2] + ssum[3]);   // (ordered by the barrier above)
}

__global__ void gradient_sum_kernel(const double *__restrict__ gsplit, int ns, int HC, const Status *__restrict__ status,
                                    double *__restrict__ gpart)
{
    if (status->early) return;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= HC) return;
    double s = gsplit[t];
    for (int i = 1; i < ns; i++) s += gsplit[(int64_t)i * HC + t];
    gpart[t] = s;
}

// A store into the mapped host block (fine-grained host memory, not cached in L2): system scope,
// so it leaves the GPU when issued and counts on this wave's vmcnt until host memory has it.
__device__ __forceinline__ void pub(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// The host block is complete: every thread waits for its own block stores (pub) to be acknowledged,
// then one store of the update's sequence number, which the host polls (no event behind the finish
// kernel: an event record delayed the next kernel on the stream by ~6 us).  No system-scope release:
// its L2 write-back is for the device-memory stores, which only later kernels on the stream read.
// Call from every thread of the block.
__device__ __forceinline__ void publish_block(const FinishArgs &a)
{
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        // every thread has read this update's wait-timeout count (update_wait_timeouts): reset it
        // for the next rollout launch (stream-ordered after this kernel)
        a.status_w->wait_timeouts = 0;
        if (a.wait_local) *a.wait_local = 0.0;
        __hip_atomic_store(a.out + a.H * a.C + 6, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The softmin normaliser sum_r e_r from weights_gradient_kernel's GRAD_SPLIT partials, fixed order.
__device__ __forceinline__ double softmin_total(const Status &st)
{
    double t = st.tsplit[0];
#pragma unroll
    for (int i = 1; i < GRAD_SPLIT; i++) t += st.tsplit[i];
    return t;
}

// In-launch waits of this update's rollout launch that gave up (fr_coop.hip note_wait_timeout):
// every rank's when sharded over RCCL (the all-reduced cost slot R), else this handle's.  Nonzero
// means some rows' costs were never written, so the update fails the way a throwing optimise()
// does (mppi.cpp:369-370): no gradient step, no smoothing, U* not published, no filter().
__device__ __forceinline__ int update_wait_timeouts(const FinishArgs &a)
{
    return a.wait_all ? (int)*a.wait_all : a.status->wait_timeouts;
}

// U* += step * gradient; Savitzky-Golay; clamp (mppi.cpp:421-447).  One workgroup.
// SG: one thread per control dimension runs its MovingExtendedWindow (filter.cpp:19-116).
__device__ __forceinline__ void finish_block(const FinishArgs &a, int &sg_err)
{
    const Status &stt = *a.status;
    const int HC = a.H * a.C;
    const int wt = update_wait_timeouts(a);
    if (threadIdx.x == 0) sg_err = 0;
    __syncthreads();
    if (!stt.early && !wt) {
    const double total = softmin_total(stt);
    if (threadIdx.x == 0) a.status_w->total = total;
    for (int t = threadIdx.x; t < HC; t += blockDim.x) {
        double g;
        if (a.ns > 0) {   // stage 2 of the gradient, fixed order
            g = a.gsplit[t];
            for (int i = 1; i < a.ns; i++) g += a.gsplit[(int64_t)i * HC + t];
        } else {
            g = a.gpart[t];
        }
        g /= total;   // sum_r e_r eps_r / sum_r e_r
        a.gradient[t] = g;
        a.Ushift[t] += g * a.gradient_step;
    }
    __syncthreads();
    if (a.sg_window > 0) {
        const int c = threadIdx.x;
        if (c < a.C) {
            const int w = a.sg_window;
            const int W = a.H + 2 * w + 1;
            double *uu = a.sg_uu + (int64_t)c * W;
            double *tt = a.sg_tt + (int64_t)c * W;
            int64_t start_idx = a.sg_start[c];
            double last_trim = a.sg_last_trim[c];
            const double t0 = a.t0;
            int err = 0;
            // trim(t0)
            if (t0 < last_trim) err = 1;
            if (!err) {
                last_trim = t0;
                int64_t trim_idx = start_idx;
                for (int64_t i = 0; i < start_idx; i++)
                    if (tt[i] >= t0) { trim_idx = i; break; }
                const int64_t offset = trim_idx - w;
                if (offset > 0) {   // std::rotate left by offset, then extend with the last kept value
                    for (int64_t i = 0; i < W - offset; i++) { tt[i] = tt[i + offset]; uu[i] = uu[i + offset]; }
                    const double tl = tt[W - offset - 1], ul = uu[W - offset - 1];
                    for (int64_t i = W - offset; i < W; i++) { tt[i] = tl; uu[i] = ul; }
                }
                start_idx = w;
                tt[start_idx] = t0;
                // add_measurement for each step
                for (int k = 0; k < a.H && !err; k++) {
                    const double tk = step_time(t0, k, a.dt);
                    if (tk < tt[start_idx]) { err = 1; break; }
                    const double v = a.Ushift[k * a.C + c];
                    uu[start_idx] = v;
                    tt[start_idx] = tk;
                    for (int64_t i = start_idx + 1; i < W; i++) { uu[i] = v; tt[i] = tk; }
                    start_idx++;
                }
                // apply for each step: extract centred at lower_bound(t), then set(idx - 1)
                for (int k = 0; k < a.H && !err; k++) {
                    const double tk = step_time(t0, k, a.dt);
                    int64_t lo = 0, hi = W;
                    while (lo < hi) {
                        const int64_t mid = (lo + hi) / 2;
                        if (tt[mid] < tk) lo = mid + 1;
                        else hi = mid;
                    }
                    const int64_t idx = lo;
                    double res = a.sg_weights[0] * uu[idx - w];
                    for (int j = 1; j < 2 * w + 1; j++) res += a.sg_weights[j] * uu[idx - w + j];
                    res = res / 1.0;
                    a.Ushift[k * a.C + c] = res;
                    uu[idx - 1] = res;
                }
            }
            a.sg_start[c] = start_idx;
            a.sg_last_trim[c] = last_trim;
            if (err) sg_err = 1;
        }
        __syncthreads();
    }
    if (a.control_bound) {
        for (int t = threadIdx.x; t < HC; t += blockDim.x) {
            const int c = t % a.C;
            double u = a.Ushift[t];
            u = smin(u, a.cmax[c]);
            u = smax(u, a.cmin[c]);
            a.Ushift[t] = u;
        }
    }
    }
    __syncthreads();
    // publish (mppi.cpp:178-182): U* <- U*_shifted unless the update threw
    const bool ok = !stt.all_nan && !sg_err && !wt;
    for (int t = threadIdx.x; t < HC; t += blockDim.x) {
        const double v = ok ? a.Ushift[t] : a.U[t];
        if (ok) a.U[t] = v;
        pub(a.out + t, v);
    }
    if ((int)threadIdx.x < a.X) a.x0_opt[threadIdx.x] = a.x0[threadIdx.x];
    for (int64_t i = threadIdx.x; i < a.rank_n; i += blockDim.x) a.rank_zero[i] = 0;   // for rank_tiled_kernel
    if (threadIdx.x == 0) {
        a.status_w->sg_error = sg_err || wt;   // read by the filter() row as "the update threw"
        pub(a.out + HC + 0, *a.opt_cost);
        pub(a.out + HC + 1, (double)stt.all_nan);
        pub(a.out + HC + 2, (double)stt.early);
        pub(a.out + HC + 3, (double)sg_err);
        pub(a.out + HC + 4, stt.minimum);
        pub(a.out + HC + 5, stt.maximum);
        pub(a.out + HC + 7, (double)wt);
    }
}

__global__ __launch_bounds__(256) void finish_kernel(FinishArgs a)
{
    __shared__ int sg_err;
    finish_block(a, sg_err);
    if (a.stats_reset) mppi_sample::reset_cost_stats(a.stats_reset, threadIdx.x);
    publish_block(a);
}

// finish() without the Savitzky-Golay filter, one U* element per thread.  Every load of the block's
// first (at H C <= 1024 its only) output is issued in one batch with the status words, the wait
// count, the optimal cost and the state, before anything waits: the block makes one dependent
// memory trip behind its arguments where finish_block makes five (gradient splits, U*_shifted, the
// bounds, U*, then the host block).  (Round 6: the wait count's source and thread 0's optimal cost
// behind branches, and the outputs' loads inside the loop behind the normaliser's sum, had made it
// four scalar round trips before the partials were requested.)
__global__ __launch_bounds__(1024) void finish_flat_kernel(FinishArgs a)
{
    const int HC = a.H * a.C, t0 = threadIdx.x;
    const int nsp = a.ns > 0 ? a.ns : 1;
    const double *__restrict__ gs = a.ns > 0 ? a.gsplit : a.gpart;
    double *__restrict__ Us = a.Ushift;
    double *__restrict__ U = a.U;
    const bool split8 = nsp == GRAD_SPLIT;   // the usual split: its partials loaded together, added in order
    const int tf = t0 < HC ? t0 : 0;
    const int cf = tf % a.C;
    double pf[GRAD_SPLIT];
#pragma unroll
    for (int i = 0; i < GRAD_SPLIT; i++) pf[i] = gs[(int64_t)(split8 ? i : 0) * HC + tf];
    const double uf = Us[tf], uof = U[tf], hif = a.cmax[cf], lof = a.cmin[cf];
    const Status stt = *a.status;   // the status words, the normaliser partials, min / max
    const double wa = *(a.wait_all ? a.wait_all : a.opt_cost);   // (a select of sources, not a branch)
    const double oc = *a.opt_cost;
    const double x0 = t0 < a.X ? a.x0[t0] : 0.0;
    const int wt = a.wait_all ? (int)wa : stt.wait_timeouts;   // update_wait_timeouts
    const bool upd = !stt.early && !wt, ok = !stt.all_nan && !wt;   // no filter: no SG error
    double total = stt.tsplit[0];   // softmin_total
#pragma unroll
    for (int i = 1; i < GRAD_SPLIT; i++) total += stt.tsplit[i];
    auto finish = [&](int t, double g, double u, double uo, double hi, double lo) {
        g /= total;   // sum_r e_r eps_r / sum_r e_r
        if (upd) {
            a.gradient[t] = g;
            u += g * a.gradient_step;
            if (a.control_bound) {
                u = smin(u, hi);
                u = smax(u, lo);
            }
            Us[t] = u;
        }
        const double v = ok ? u : uo;
        if (ok) U[t] = v;
        pub(a.out + t, v);
    };
    auto partials = [&](int t) {   // another split count, or outputs past the first: loaded here
        double g = gs[t];
        for (int i = 1; i < nsp; i++) g += gs[(int64_t)i * HC + t];
        return g;
    };
    if (t0 < HC) {
        double g;
        if (split8) {
            g = pf[0];
#pragma unroll
            for (int i = 1; i < GRAD_SPLIT; i++) g += pf[i];
        } else {
            g = partials(t0);
        }
        finish(t0, g, uf, uof, hif, lof);
    }
    for (int t = t0 + (int)blockDim.x; t < HC; t += blockDim.x) {
        const int c = t % a.C;
        finish(t, partials(t), Us[t], U[t], a.cmax[c], a.cmin[c]);
    }
    if ((int)threadIdx.x < a.X) a.x0_opt[threadIdx.x] = x0;
    for (int64_t i = threadIdx.x; i < a.rank_n; i += blockDim.x) a.rank_zero[i] = 0;   // for rank_tiled_kernel
    if (threadIdx.x == 0) {
        a.status_w->sg_error = wt != 0;   // read by the filter() row as "the update threw"
        if (upd) a.status_w->total = total;
        pub(a.out + HC + 0, oc);
        pub(a.out + HC + 1, (double)stt.all_nan);
        pub(a.out + HC + 2, (double)stt.early);
        pub(a.out + HC + 3, 0.0);
        pub(a.out + HC + 4, stt.minimum);
        pub(a.out + HC + 5, stt.maximum);
        pub(a.out + HC + 7, (double)wt);
    }
    if (a.stats_reset) mppi_sample::reset_cost_stats(a.stats_reset, threadIdx.x);
    publish_block(a);
}




// finish() with the Savitzky-Golay filter (configs[4]), one wave per control dimension with its
// MovingExtendedWindow (filter.cpp:19-116) staged in LDS.  finish_block runs the reference's loops
// literally on one thread per dimension over global memory: its add_measurement refills the whole
// window tail per step (O(H W) stores) and apply() binary-searches per step, 0.89 ms at H = 128.
// Here, per dimension:
//   trim(t0)        first index >= t0 by ballots; the left rotation (tail repeating the last kept
//                   element) as one gather new[i] = old[min(i + offset, W - 1)].
//   add_measurement the window's final state in one pass: uu[w + k] = U*_k, tt[w + k] = t_k, and
//                   the last measurement repeated past w + H (the reference's successive fills).
//                   Its "older than the new time" check cannot fire: t_k = t0 + k dt is monotone
//                   and trim just set tt[w] = t0.
//   apply           with lower_bound(t_k) = w + k for every k (checked: tt[w + k - 1] < t_k), step
//                   k reads uu[k .. k + 2w] and then writes its output over uu[w + k - 1].  Terms
//                   j >= w - 1 are measurements or old history no step has overwritten yet, so
//                   P_k = sum_{j >= w-1} wt_j uu[k + j] is formed for all k at once; the rest is the
//                   order-(w-1) recurrence res_k = P_k + sum_{j < w-1} wt_j z(k + j), with z(p) the
//                   output written at p (res_{p-w+1}) or, before the first, the old history uu[p].
//                   Any other lower_bound pattern falls back to the literal loop in LDS.
// Sums are associated differently from the reference's left-to-right loop (rounding only).
constexpr int SGK_MAXW = 384;   // largest window W = H + 2w + 1 this kernel stages (else finish_kernel)

__device__ __forceinline__ int lds_lower_bound(const double *tt, int W, double t)
{
    int lo = 0, hi = W;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tt[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

constexpr int SGK_ZM = 15;   // w - 1 <= SGK_ZM: the recurrence's outputs in registers

__global__ __launch_bounds__(1024) void sg_finish_kernel(FinishArgs a)
{
    extern __shared__ double sg_lds[];   // per dimension: uu[W], tt[W], res[H]; then wt[2w + 1]
    __shared__ int sg_err, sg_mode[16];  // per dimension: 0 trim error, 1 literal loop, 2 recurrence
    const Status &stt = *a.status;
    const int H = a.H, C = a.C, HC = H * C, w = a.sg_window, W = H + 2 * w + 1, nw = 2 * w + 1;
    const int t = threadIdx.x, c = t >> 6, l = t & 63;
    const int wt = update_wait_timeouts(a);
    const bool upd = !stt.early && !wt;   // optimise() returned before the filter (mppi.cpp:373-375)
    double *wl = sg_lds + (int64_t)C * (2 * W + H);
    if (t == 0) sg_err = 0;
    if (t < nw) wl[t] = a.sg_weights[t];
    if (upd) {
        const double total = softmin_total(stt);
        if (t == 0) a.status_w->total = total;
        for (int i = t; i < HC; i += blockDim.x) {
            double g;
            if (a.ns > 0) {   // stage 2 of the gradient, fixed order
                g = a.gsplit[i];
                for (int k = 1; k < a.ns; k++) g += a.gsplit[(int64_t)k * HC + i];
            } else {
                g = a.gpart[i];
            }
            g /= total;   // sum_r e_r eps_r / sum_r e_r
            a.gradient[i] = g;
            a.Ushift[i] += g * a.gradient_step;
        }
    }
    __syncthreads();
    double *uu = sg_lds + (int64_t)(c < C ? c : 0) * (2 * W + H), *tt = uu + W, *res = tt + W;
    double *guu = a.sg_uu + (int64_t)c * W, *gtt = a.sg_tt + (int64_t)c * W;
    const double t0 = a.t0;
    if (upd && c < C) {   // phase 1, wave c: trim + add_measurement, then P_k or the literal loop
        for (int i = l; i < W; i += 64) {
            uu[i] = guu[i];
            tt[i] = gtt[i];
        }
        const int start_idx = (int)a.sg_start[c];
        if (t0 < a.sg_last_trim[c]) {   // trim: "Resetting the window back in the past." - untouched
            if (l == 0) { sg_mode[c] = 0; sg_err = 1; }
        } else {
            __builtin_amdgcn_wave_barrier();
            int trim_idx = start_idx;
            for (int base = 0; base < start_idx; base += 64) {
                const int i = base + l;
                const uint64_t b = __ballot(i < start_idx && tt[i] >= t0);
                if (b) {
                    trim_idx = base + __builtin_ctzll(b);
                    break;
                }
            }
            const int offset = trim_idx - w;
            if (offset > 0) {
                double ru[SGK_MAXW / 64], rt[SGK_MAXW / 64];
#pragma unroll
                for (int m = 0; m < SGK_MAXW / 64; m++) {
                    const int i = l + 64 * m, src = (i + offset < W) ? i + offset : W - 1;
                    if (i < W) { ru[m] = uu[src]; rt[m] = tt[src]; }
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int m = 0; m < SGK_MAXW / 64; m++) {
                    const int i = l + 64 * m;
                    if (i < W) { uu[i] = ru[m]; tt[i] = rt[m]; }
                }
            }
            for (int i = w + l; i < W; i += 64) {   // the H measurements, then the last one repeated
                const int k = (i - w < H) ? i - w : H - 1;
                uu[i] = a.Ushift[k * C + c];
                tt[i] = step_time(t0, k, a.dt);
            }
            __builtin_amdgcn_wave_barrier();
            bool ok = w - 1 <= SGK_ZM;   // and lower_bound(t_k) == w + k for every k
            for (int k = l; k < H; k += 64) ok = ok && tt[w + k - 1] < step_time(t0, k, a.dt);
            if (__ballot(!ok) == 0) {
                for (int k = l; k < H; k += 64) {   // P_k: the terms no earlier step has overwritten
                    double p = 0.0;
                    for (int j = w - 1; j < nw; j++) p += wl[j] * uu[k + j];
                    res[k] = p;
                }
                if (l == 0) sg_mode[c] = 2;
            } else if (l == 0) {   // the literal loop (filter.cpp:92-110)
                sg_mode[c] = 1;
                for (int k = 0; k < H; k++) {
                    const int idx = lds_lower_bound(tt, W, step_time(t0, k, a.dt));
                    double r = wl[0] * uu[idx - w];
                    for (int j = 1; j < nw; j++) r += wl[j] * uu[idx - w + j];
                    a.Ushift[k * C + c] = r;
                    uu[idx - 1] = r;
                }
            }
        }
    }
    __syncthreads();
    if (upd && t < C && sg_mode[t] == 2) {   // phase 2, lane d of wave 0: dimension d's recurrence
        // z: the last w - 1 window entries below the current step's P_k terms, right-aligned (the
        // newest, output k - 1, in z[ZM - 1]); slots left of the window have weight 0
        const int d = t, nz = w - 1;
        double *uud = sg_lds + (int64_t)d * (2 * W + H), *resd = uud + 2 * W;
        double z[SGK_ZM], wr[SGK_ZM];
#pragma unroll
        for (int j = 0; j < SGK_ZM; j++) {
            const int q = j - (SGK_ZM - nz);   // window offset of slot j
            wr[j] = q >= 0 ? wl[q] : 0.0;
            z[j] = q >= 0 ? uud[q] : 0.0;      // old history uu[0 .. w - 2]
        }
        for (int k = 0; k < H; k++) {
            // four partial sums: output k - 1 (slot ZM - 1) is three dependent ops from output k
            double ac[4] = {resd[k], 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j < SGK_ZM; j++) ac[j & 3] = __builtin_fma(wr[j], z[j], ac[j & 3]);
            const double acc = (ac[0] + ac[1]) + (ac[2] + ac[3]);
            resd[k] = acc;
#pragma unroll
            for (int j = 0; j + 1 < SGK_ZM; j++) z[j] = z[j + 1];
            z[SGK_ZM - 1] = acc;
        }
    }
    __syncthreads();
    if (upd && c < C && sg_mode[c] != 0) {   // phase 3, wave c: outputs into U* and the window
        if (sg_mode[c] == 2) {
            for (int k = l; k < H; k += 64) {   // output k over the window at w + k - 1
                a.Ushift[k * C + c] = res[k];
                uu[w + k - 1] = res[k];
            }
            __builtin_amdgcn_wave_barrier();
        }
        for (int i = l; i < W; i += 64) {
            guu[i] = uu[i];
            gtt[i] = tt[i];
        }
        if (l == 0) {
            a.sg_start[c] = w + H;
            a.sg_last_trim[c] = t0;
        }
    }
    __syncthreads();
    if (upd && a.control_bound) {
        for (int i = t; i < HC; i += blockDim.x) {
            const int cc = i % C;
            a.Ushift[i] = smax(smin(a.Ushift[i], a.cmax[cc]), a.cmin[cc]);
        }
    }
    __syncthreads();
    // publish (mppi.cpp:178-182): U* <- U*_shifted unless the update threw
    const int err = sg_err;
    const bool ok = !stt.all_nan && !err && !wt;
    for (int i = t; i < HC; i += blockDim.x) {
        const double v = ok ? a.Ushift[i] : a.U[i];
        if (ok) a.U[i] = v;
        pub(a.out + i, v);
    }
    if (t < a.X) a.x0_opt[t] = a.x0[t];
    for (int64_t i = t; i < a.rank_n; i += blockDim.x) a.rank_zero[i] = 0;   // for rank_tiled_kernel
    if (t == 0) {
        a.status_w->sg_error = err || wt;   // read by the filter() row as "the update threw"
        pub(a.out + HC + 7, (double)wt);
        pub(a.out + HC + 0, *a.opt_cost);
        pub(a.out + HC + 1, (double)stt.all_nan);
        pub(a.out + HC + 2, (double)stt.early);
        pub(a.out + HC + 3, (double)err);
        pub(a.out + HC + 4, stt.minimum);
        pub(a.out + HC + 5, stt.maximum);
    }
    if (a.stats_reset) mppi_sample::reset_cost_stats(a.stats_reset, t);
    publish_block(a);
}

// ---------------------------------------------------------------------------------------------
// Launch wrappers (host).
// ---------------------------------------------------------------------------------------------
namespace mppi_eng {

hipError_t launch_rank(const double *cost, int64_t S, int *rank, uint64_t *sorted, hipStream_t s)
{
    if (S <= 0) return hipSuccess;
    if (S <= RANK_TILED_MAX) {   // rank[] zeroed by the finish kernel (or at create)
        const unsigned nb = (unsigned)((S + RANK_T - 1) / RANK_T);
        hipLaunchKernelGGL(rank_tiled_kernel, dim3(nb, nb), dim3(RANK_T), 0, s, cost, S, rank);
        return hipGetLastError();
    }
    const unsigned nch = (unsigned)((S + RANK_T - 1) / RANK_T);
    hipLaunchKernelGGL(rank_chunk_kernel, dim3(nch), dim3(RANK_T), 0, s, cost, S, rank, sorted);
    if (nch > 1)
        hipLaunchKernelGGL(rank_merge_kernel, dim3(nch, (nch + RANK_G - 1) / RANK_G), dim3(RANK_T), 0, s, cost, S, rank,
                           (const uint64_t *)sorted);
    return hipGetLastError();
}

hipError_t launch_sample(const SampleArgs &a, bool tdiag, hipStream_t s)
{
    if (a.count <= 0 && a.sp.shift_by <= 0) return hipSuccess;
    const int nb = tdiag ? (a.C + 3) / 4 : 1;
    const int64_t nx = (a.count * nb + 255) / 256;
    const dim3 grid((unsigned)(nx > 0 ? nx : 1), (unsigned)a.H);
    if (a.C == FR_C) {
        if (tdiag) hipLaunchKernelGGL((sample_kernel<FR_C, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((sample_kernel<FR_C, false>), grid, dim3(256), 0, s, a);
    } else if (a.C == 3) {
        if (tdiag) hipLaunchKernelGGL((sample_kernel<3, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((sample_kernel<3, false>), grid, dim3(256), 0, s, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_pm_rollout(const PmRolloutArgs &a, hipStream_t s)
{
    const unsigned nb = (unsigned)((a.count + 255) / 256);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(pm_rollout_kernel, dim3(nb), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_weights_gradient(const WGradArgs &a, double *gpart, bool sum_splits, hipStream_t s)
{
    // C = FR_C: WG_KPB steps per workgroup (weights_gradient_kernel)
    const dim3 grid(a.C == FR_C ? (unsigned)((a.H + WG_KPB - 1) / WG_KPB) : (unsigned)a.H, GRAD_SPLIT);
    if (a.C != FR_C && a.C != 3) return hipErrorInvalidValue;
    if (a.R > SM_LARGE_R) {
        hipLaunchKernelGGL(softmin_minmax_kernel, dim3(SM_NB), dim3(256), 0, s, a);
        hipLaunchKernelGGL(softmin_exp_kernel, dim3(SM_NB), dim3(256), 0, s, a);
        if (a.C == FR_C) hipLaunchKernelGGL((weights_gradient_kernel<FR_C, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((weights_gradient_kernel<3, true>), grid, dim3(256), 0, s, a);
    } else {
        if (a.C == FR_C) hipLaunchKernelGGL((weights_gradient_kernel<FR_C, false>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((weights_gradient_kernel<3, false>), grid, dim3(256), 0, s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !sum_splits) return e;   // unsharded: the finish kernel adds the splits itself
    const int HC = a.H * a.C;
    hipLaunchKernelGGL(gradient_sum_kernel, dim3((HC + 255) / 256), dim3(256), 0, s, a.gsplit, GRAD_SPLIT, HC,
                       (const Status *)a.status, gpart);
    return hipGetLastError();
}

int graph_kernel_kind(const void *f)
{
    auto is = [f](const void *k) { return f == k; };
    if (is((const void *)&weights_gradient_kernel<FR_C, false>) || is((const void *)&weights_gradient_kernel<FR_C, true>) ||
        is((const void *)&weights_gradient_kernel<3, false>) || is((const void *)&weights_gradient_kernel<3, true>) ||
        is((const void *)&softmin_minmax_kernel) || is((const void *)&softmin_exp_kernel))
        return GK_WGRAD;
    if (is((const void *)&finish_flat_kernel) || is((const void *)&sg_finish_kernel) || is((const void *)&finish_kernel))
        return GK_FINISH;
    if (is((const void *)&rank_draw_kernel<FR_C>)) return GK_RANKDRAW;
    return GK_OTHER;
}

hipError_t launch_finish(const FinishArgs &a, hipStream_t s)
{
    const int W = a.H + 2 * a.sg_window + 1;
    const size_t lds = ((size_t)a.C * (2 * W + a.H) + 2 * a.sg_window + 1) * sizeof(double);
    if (a.sg_window > 0 && W <= SGK_MAXW && a.C <= 16 && lds <= 65536) {
        hipLaunchKernelGGL(sg_finish_kernel, dim3(1), dim3(64 * (a.C > 4 ? a.C : 4)), lds, s, a);
    } else if (a.sg_window > 0) {
        hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(finish_flat_kernel, dim3(1), dim3(1024), 0, s, a);
    }
    return hipGetLastError();
}


}  // namespace mppi_eng
