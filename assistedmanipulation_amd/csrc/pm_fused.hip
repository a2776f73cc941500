// pm_fused.hip — one launch per point-mass update (BASELINE configs[1], 1024 x 32).
//
// The point-mass update (the a16 bring-up plugin: quadratic cost, ~25 flops per rollout-step) has
// no arithmetic to speak of; in five launches (sample, rollouts, weights + gradient, finish, rank)
// its time was the launches' fixed costs and their dependent memory trips.  Here one grid of
// 256-thread workgroups, each owning PR rollouts (16 up to 1024 rollouts, 64 above), runs the whole
// of Trajectory::update (mppi.cpp:154-187) with one grid barrier:
//
//   phase A  sample (mppi.cpp:189-270): the block's eps columns into LDS (and the eps tensor):
//            rollout 0 zero, rollout 1 = -U*, kept rollouts the previous eps shifted, the rest
//            Philox by (rollout, step) - drawn ahead by the previous launch when it could; U*
//            shifted.  Every candidate source (kept, drawn ahead) is loaded in one batch with the
//            rank, so the phase is one memory trip; then one wave rolls the rollouts out of LDS
//            (mppi.cpp:272-342) and folds the costs' min / max / count into the CostStats slots
//            (exact key atomics).
//   barrier  every block's costs and statistics are final.
//   phase B  optimise (mppi.cpp:344-418): e_r of the block's rollouts and its partial gradient
//            sum_r e_r eps_r over its PR rollouts (fixed order), written through to L2 (sc1) for
//            the last block to arrive (agent-scope ticket), which stages every block's partials in
//            LDS in one batch of loads, adds them in block order, steps U*, clamps and publishes
//            the host block (mppi.cpp:421-447, 178-182).
//   tail     while the host turns around: the stable rank of the block's rollouts (the next
//            update's keep-best) and the next update's Philox draws of its rollouts.
//
// filter() (mppi.cpp:450-479) of the published U* is left pending, as the cooperative rollout
// launch leaves it: the next launch runs it at the end of block 0's tail, from the U* and state it
// copied at entry (behind the publish, off the update's chain), or a read of the optimal cost runs
// it first (wait_optimal).
//
// Cross-block hand-offs follow MI355X_MICROARCH.md's measured forms: payloads stored sc1
// (write-through) and drained with vmcnt(0) before an agent-scope atomic add; readers poll with
// sc1 loads and load the payload with sc1 loads, issued together.  Every wait is bounded: a block
// that gives up counts it in Status::wait_timeouts, and the update then fails like the rollout
// launch's waits.  A rollout's arithmetic is pm_rollout_kernel's (kernels.hip) operation for
// operation, so the costs are bit-identical to the five-launch path on the same operands; the
// gradient and the normaliser are summed in another order (rounding only).
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

constexpr int PT = PM_FUSED_THREADS;   // threads per block
constexpr int PC = 3;                  // control dimension of the point mass
// a store into the mapped host block, system scope (kernels.hip pub)
__device__ __forceinline__ void pub(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
constexpr int BAR_SPINS = 1 << 22;     // about a second of s_sleep 1
constexpr int IB = 8;                  // phase A items per thread per batch of loads
constexpr int SB = 32;              // sc1 loads per thread per batch (the finisher's and the rank's staging)

__device__ __forceinline__ double ld_sc1(const double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// the rank's order (kernels.hip cost_key): order-preserving, -0 = +0, NaN last
__device__ __forceinline__ uint64_t rank_key(double c)
{
    return isnan(c) ? ~0ull : mppi_dev::cost_order_key(c);
}

// the doubles of the eps rows [PR][H C + 1] and the rollouts' control part [H][PR][4] behind them
// (pm_rollout_pre), which the finisher reuses for every block's partials once the rollouts are done
__host__ __device__ inline int64_t pm_region(int PR, int HC, int64_t nb)
{
    const int H = HC / PC;
    const int64_t e = (int64_t)PR * (HC + 1) + 4 * (int64_t)PR * H, p = nb * HC + nb;
    return e > p ? e : p;
}

// Philox eps of (rollout g, step k) for update `upd`: sample_device.hpp's diagonal piece 0, three
// components used
__device__ __forceinline__ void philox_eps(const PmFusedArgs &a, int64_t g, int k, uint64_t upd, double *e)
{
    const int64_t draw = mppi_sample::philox_index(g, k, a.H);
    const mppi_dev::u32x4 ctr{(uint32_t)draw, (uint32_t)((uint64_t)draw >> 32), (uint32_t)upd, 0u};
    const mppi_dev::u32x4 r = mppi_dev::philox4x32_10(ctr, (uint32_t)a.sp.seed, (uint32_t)(a.sp.seed >> 32));
    float z[4];
    mppi_dev::box_muller(r.x, r.y, z[0], z[1]);
    mppi_dev::box_muller(r.z, r.w, z[2], z[3]);
#pragma unroll
    for (int c = 0; c < PC; c++) e[c] = a.tdv[c] * (double)z[c];
}

// pm_rollout_kernel's horizon (kernels.hip pm_steps): pm_model.hpp's control and state parts in the
// same order, so the costs are bit-identical to the five-launch path; eps row k at eps[k * PC]
// (unused when optimal).  No branch per step: a NaN step cost leaves J NaN to the end, which is the
// reference's NaN rollout cost (mppi.cpp:331-334); the states it integrates past that point are
// never read.  (A step cost of +inf followed by -inf, which the reference would sum to NaN and not
// stop on, is NaN here as well.)  The update's rollouts take the control part from the block's
// precomputed table (pm_rollout_pre); this form runs the folded filter() row.
__device__ __forceinline__ double pm_rollout(const PmFusedArgs &a, const double *x0, const double *Lus, const double *Lgm,
                                             const double *eps, bool optimal)
{
    const DevPointMass &P = a.pm;
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = x0[i];
    double J = 0.0;
#pragma unroll 4
    for (int k = 0; k < a.H; k++) {
        double u[3], dv[3], cu;
#pragma unroll
        for (int c = 0; c < 3; c++) u[c] = Lus[k * PC + c] + (optimal ? 0.0 : eps[k * PC + c]);
        pm_control_step(P, u, a.dt, dv, cu);
        pm_state_step(P, x, dv, cu, Lgm[k], a.dt, J);
    }
    return J;
}

// The rollout of lane l through the horizon, its control part read from Lpre [H][PR][4] (dv0, dv1,
// dv2, cu per step, formed by the whole block in parallel): 18 fp64 operations per step on the chain
template <int PR>
__device__ __forceinline__ double pm_rollout_pre(const PmFusedArgs &a, const double *x0, const double *Lgm, const double *Lpre,
                                                 int l)
{
    const DevPointMass &P = a.pm;
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = x0[i];
    double J = 0.0;
#pragma unroll 8
    for (int k = 0; k < a.H; k++) {
        const double2 p01 = *reinterpret_cast<const double2 *>(Lpre + (k * PR + l) * 4);
        const double2 p23 = *reinterpret_cast<const double2 *>(Lpre + (k * PR + l) * 4 + 2);
        const double dv[3] = {p01.x, p01.y, p23.x};
        pm_state_step(P, x, dv, p23.y, Lgm[k], a.dt, J);
    }
    return J;
}

// p[0] + p[s] + ... + p[(n - 1) s] from 0.0 in index order (LDS), eight reads in flight at a time
__device__ __forceinline__ double sum_in_order(const double *p, int n, int s)
{
    double acc = 0.0;
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = p[(i + u) * s];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u];
    }
    for (; i < n; i++) acc += p[i * s];
    return acc;
}

// p[0] + p[ps] + ... and q[0] + q[qs] + ..., n terms each from 0.0 in index order: the two chains
// interleaved, sixteen reads of each in flight at a time
__device__ __forceinline__ void sum2_in_order(const double *p, int ps, const double *q, int qs, int n, double &a, double &b)
{
    a = 0.0;
    b = 0.0;
    int i = 0;
    for (; i + 16 <= n; i += 16) {
        double v[16], w[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            v[u] = p[(i + u) * ps];
            w[u] = q[(i + u) * qs];
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            a += v[u];
            b += w[u];
        }
    }
    for (; i < n; i++) {
        a += p[i * ps];
        b += q[i * qs];
    }
}

}  // namespace

// LDS (doubles): U*_shifted [H C], gamma [H], the block's costs [PR] and e_r [PR], the rank's keys
// [R - 2], the eps rows [PR][ES] (ES = H C + 1: the rollout wave's lanes then read distinct banks;
// the finisher's staged partials after phase B), the rank's partial counts [QD - 1][PR] (ints)
template <int PR>
__global__ __launch_bounds__(PT) void pm_update_kernel(PmFusedArgs a)
{
    static_assert(PT % PR == 0 && PR <= 64, "a thread's phase A items share one rollout; one wave rolls them out");
    constexpr int QD = PT / PR;   // threads per rollout (phase A items, the rank's key quarters)
    extern __shared__ double lds[];
    const int H = a.H, HC = H * PC, ES = HC + 1, t = threadIdx.x, w = t >> 6, l = t & 63;
    const int S = (int)(a.R - 2);
    const int b = blockIdx.x, nb = gridDim.x;
    double *Lus = lds;
    double *Lgm = Lus + HC;
    double *Lcost = Lgm + H;
    double *Le = Lcost + PR;
    uint64_t *Lkey = reinterpret_cast<uint64_t *>(Le + PR);
    double *Leps = reinterpret_cast<double *>(Lkey + S);
    int *Lcnt = reinterpret_cast<int *>(Leps + pm_region(PR, HC, nb));
    // the previous update's U* [HC] and state [6] for the folded filter()
    double *LUf = reinterpret_cast<double *>(Lcnt + (QD - 1) * PR);
    // the rollouts' control part per step, [H][PR][4] (pm_rollout_pre), behind the eps rows in the
    // finisher's staging region (free until the rollouts are done; PR ES is even, so 16-byte aligned
    // as Leps is)
    double *Lpre = Leps + PR * ES;
    __shared__ int s_last;
    const int64_t r0 = (int64_t)b * PR;
    const SampleParams &P = a.sp;
    const double *Uprev = a.U;   // U* as the previous update published it
    const unsigned target = a.epoch * (unsigned)nb;
    auto stamp = [&](int i) {   // diagnostics: one clock stamp per block and phase
        if (a.stamps && t == 0) a.stamps[b * PM_STAMPS + i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // ---- phase A: sample (mppi.cpp:189-270) ----
    // every item (step k) of this thread belongs to rollout g = r0 + rl (PT % PR == 0)
    const int rl = t % PR;
    const int64_t g = r0 + rl;
    const bool row = g < a.R;
    const int64_t gc = row ? g : 0;   // a valid address for the speculative loads of rows past R
    // loaded unconditionally and first used by the items (rollouts >= 2): its wait falls after the
    // eps batch is issued
    const int rank = a.rank[gc];
    const int keep = P.keep < 0x7FFFFFFF ? (int)P.keep : 0x7FFFFFFF;
    auto us_at = [&](int i) {   // U*_shifted (mppi.cpp:197-207); unshifted, as last left
        const int k = i / PC, c = i - k * PC;
        return P.shift_by > 0 ? (k < P.shifted ? Uprev[(k + P.shift_by) * PC + c] : Uprev[(H - 1) * PC + c]) : a.Us[i];
    };
    // loaded here, stored to LDS after the eps batch: their loads travel with it
    const double us_t = t < HC ? us_at(t) : 0.0, gm_t = t < H ? a.steps[t].gamma_k : 0.0;
    // the finisher's operands of its first output (U* as published, the bounds), loaded with the
    // batch: behind the partial sums its publish then waits on no load (they were a memory trip of
    // the finisher's "stored" phase)
    const bool cb = t < HC && a.control_bound;
    const double uo_t = t < HC ? a.U[t] : 0.0, hi_t = cb ? a.cmax[t % PC] : 0.0, lo_t = cb ? a.cmin[t % PC] : 0.0;
    const double x0_t = t < a.X ? a.x0v[t] : 0.0;   // (its x0_opt copy)
    // and its scalar arguments into the constant cache now: loaded first behind the sums, each missed
    // it and their waits made a chain of scalar round trips there
    asm volatile("" : : "s"(a.U), "s"(a.Us), "s"(a.gradient), "s"(a.out), "s"(a.x0_opt), "s"(a.seq), "s"(a.gradient_step),
                 "s"(a.control_bound), "s"(a.status), "s"(a.stats));
    if (t == 0) s_last = 0;
    auto items = [&](int k0) {
        // both candidate sources of each item (the previous eps shifted, the draw made ahead or -U*)
        // loaded in one batch with the rank: one memory trip, whichever the rank picks
        double ep[IB][PC], en[IB][PC];
#pragma unroll
        for (int u = 0; u < IB; u++) {
            if (k0 + u * QD >= H) break;
            const int k = k0 + u * QD;
            const int kp = (P.shift_by > 0 && k < P.shifted) ? k + P.shift_by : k;
            const double *pp = a.prev + ((int64_t)kp * a.Rpad + gc) * PC;
            const double *pn = g == 1 ? Uprev + k * PC : a.noise + ((int64_t)k * a.Rpad + gc) * PC;
#pragma unroll
            for (int c = 0; c < PC; c++) {
                ep[u][c] = pp[c];
                en[u][c] = pn[c];
            }
        }
        int rk = rank;
        asm volatile("" : "+v"(rk));   // the rank's first use here, not hoisted ahead of the batch
#pragma unroll
        for (int u = 0; u < IB; u++) {
            const int k = k0 + u * QD;
            if (k >= H) break;
            double *le = Leps + rl * ES + k * PC;
            if (!row) {   // rows past R: zeros, which the gradient's fixed PR-row sum multiplies by 0
#pragma unroll
                for (int c = 0; c < PC; c++) le[c] = 0.0;
                continue;
            }
            double e[PC];
            bool store = true;
            if (g == 0) {
#pragma unroll
                for (int c = 0; c < PC; c++) e[c] = 0.0;
            } else if (g == 1) {   // m_rollouts[1].noise = -m_optimal_control
#pragma unroll
                for (int c = 0; c < PC; c++) e[c] = -1.0 * en[u][c];
            } else if (rk < keep && (P.shift_by <= 0 || k < P.shifted)) {   // kept: the previous eps, shifted
#pragma unroll
                for (int c = 0; c < PC; c++) e[c] = ep[u][c];
            } else if (a.ahead) {   // the previous launch's tail drew it into this update's buffer: in place
#pragma unroll
                for (int c = 0; c < PC; c++) e[c] = en[u][c];
                store = false;
            } else {
                philox_eps(a, g, k, P.update_index, e);
            }
            // (a global-space pointer: merged across the branches above, a generic one became
            // flat stores, which the LDS waits that follow wait for as well)
            __attribute__((address_space(1))) double *o =
                (__attribute__((address_space(1))) double *)(a.noise + ((int64_t)k * a.Rpad + g) * PC);
#pragma unroll
            for (int c = 0; c < PC; c++) le[c] = e[c];
            if (store)
#pragma unroll
                for (int c = 0; c < PC; c++) o[c] = e[c];
        }
    };
    if (H <= QD * IB)   // the common case straight-line: no loop header for the waits to merge at
        items(t / PR);
    else
        for (int k0 = t / PR; k0 < H; k0 += QD * IB) items(k0);
    if (t < HC) Lus[t] = us_t;
    for (int i = t + PT; i < HC; i += PT) Lus[i] = us_at(i);
    if (t < H) Lgm[t] = gm_t;
    for (int k = t + PT; k < H; k += PT) Lgm[k] = a.steps[k].gamma_k;
    if (b == 0 && t < a.X) a.x0_out[t] = a.x0v[t];
    // the previous update's filter() (mppi.cpp:450-479), which its launch left pending, runs in this
    // block's tail: its inputs are taken now, before this launch's finisher rewrites them - the U*
    // it published, its state (x0_opt) and whether it threw (then no filter)
    const bool fold = b == 0 && a.fold_filter && !a.status->all_nan && !a.status->sg_error;
    if (fold)
        for (int i = t; i < HC; i += PT) LUf[i] = a.U[i];
    const double fx = (fold && t < 6) ? a.fx0[t] : 0.0;
    if (fold && t < 6) LUf[HC + t] = fx;
    __syncthreads();
    stamp(1);
    // the control part of every (rollout, step) of the block, by all its threads (pm_model.hpp)
    for (int it = t; it < PR * H; it += PT) {
        const int k = it / PR, r = it - k * PR;
        double u[3], dv[3], cu;
#pragma unroll
        for (int c = 0; c < 3; c++) u[c] = Lus[k * PC + c] + Leps[r * ES + k * PC + c];
        pm_control_step(a.pm, u, a.dt, dv, cu);
        double *o = Lpre + (k * PR + r) * 4;
        *reinterpret_cast<double2 *>(o) = double2{dv[0], dv[1]};
        *reinterpret_cast<double2 *>(o + 2) = double2{dv[2], cu};
    }
    __syncthreads();
    const int64_t gr = r0 + l;   // the rollout wave's lane l
    const bool mine = w == 0 && l < PR && gr < a.R;
    double J = NAN;
    // rollouts (mppi.cpp:272-342): one lane per rollout through the horizon, the state part only.
    // (Round 4 split the state chain from the step costs - the positions through LDS, the costs by
    // all threads - and measured it slower: 28.7 against 27.6 us per update, profiles/r04/pm_split_ab/;
    // the control part needs no state, so here it is formed before the chain instead.)
    if (mine) J = pm_rollout_pre<PR>(a, a.x0v, Lgm, Lpre, l);
    stamp(11);
    if (w == 0) {
        if (mine) st_sc1(a.cost + gr, J);   // read by every block's rank (tail)
        if (l < PR) Lcost[l] = J;
        // the block's min / max / count, then one exact key atomic each into CostStats slot b % 64
        const bool ok = mine && !isnan(J);
        const unsigned long long key = ok ? mppi_dev::cost_order_key(J) : 0ull;
        const unsigned long long kn = mppi_dev::wave_umin64_dpp(ok ? key : ~0ull);
        const unsigned long long kx = mppi_dev::wave_umax64_dpp(ok ? key : 0ull);
        const double n = mppi_dev::wave_sum_dpp(ok ? 1.0 : 0.0);
        if (l == 0 && n > 0.0) {
            const int slot = b % CS_SLOTS;
            atomicMin(&a.stats->kmin[16 * slot], kn);
            atomicMax(&a.stats->kmax[16 * slot], kx);
            atomicAdd(&a.stats->count[32 * slot], (unsigned)n);
        }
        __builtin_amdgcn_s_waitcnt(0);   // the cost stores and the atomics have left this wave
    }
    __syncthreads();
    stamp(2);
    // ---- grid barrier: every block's costs and statistics are final (bounded) ----
    if (t == 0) {
        __hip_atomic_fetch_add(a.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int i = 0;
        // wrap-safe: the counter and target = epoch * nb both wrap at 2^32 (every 2^32 / nb updates)
        while ((int)(__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0 && i < BAR_SPINS) {
            __builtin_amdgcn_s_sleep(1);
            i++;
        }
        if (i == BAR_SPINS) atomicAdd(&a.status->wait_timeouts, 1);   // the update then fails
    }
    __syncthreads();
    stamp(3);
    // ---- phase B: optimise (mppi.cpp:344-418) ----
    static_assert(CS_SLOTS == 64, "one slot per lane");
    const unsigned long long kn = mppi_dev::wave_umin64_dpp(
        __hip_atomic_load(&a.stats->kmin[16 * l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const unsigned long long kx = mppi_dev::wave_umax64_dpp(
        __hip_atomic_load(&a.stats->kmax[16 * l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const unsigned cn = (unsigned)mppi_dev::wave_sum_dpp(
        (double)__hip_atomic_load(&a.stats->count[32 * l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const double mn = cn ? mppi_dev::cost_from_key(kn) : (double)INFINITY;
    const double mx = cn ? mppi_dev::cost_from_key(kx) : -(double)INFINITY;
    const bool all_nan = cn <= 1;                  // minmax_element over <= 1 element: it1 == it2 -> throw
    const double difference = mx - mn;
    const bool early = all_nan || difference < 1e-6;   // early return, weights / gradient stale (mppi.cpp:373-375)
    if (!early) {
        if (w == 0) {   // e_r of the block's rollouts, their sum in lane order
            const bool mine = l < PR && gr < a.R;
            const double c = mine ? Lcost[l] : 0.0;
            const double e = (mine && !isnan(c)) ? exp(-a.cost_scale * (c - mn) / difference) : 0.0;
            if (l < PR) Le[l] = e;
            if (mine) a.wexp[gr] = e;
            const double s = mppi_dev::wave_sum_dpp(e);
            if (l == 0) st_sc1(a.tpart + b, s);
        }
        __syncthreads();
        for (int o = t; o < HC; o += PT) {   // partial gradient: the block's rollouts in order
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < PR; r++) acc = __builtin_fma(Le[r], Leps[r * ES + o], acc);
            st_sc1(a.gpart + (int64_t)b * HC + o, acc);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);   // every wave's partial stores have left it
    __syncthreads();
    stamp(4);
    if (t == 0) {   // the last block to arrive finishes the update
        const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old + 1 == target;
    }
    __syncthreads();
    stamp(5);
    // the rank's keys (every block's tail), and in the finishing block every block's partials
    // (gradient [nb][HC], then normalisers [nb]) over the eps rows: one batch of sc1 loads, SB per
    // thread in flight at once (the other blocks stored them this launch)
    double *Lst = Leps;
    const int G = nb * HC, np = (s_last && !early) ? G + nb : 0, n = np + S;
    // with the batch, unconditionally (a branch or a loop header here makes their wait a trip)
    const int wt = __hip_atomic_load(&a.status->wait_timeouts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the partials are one array (tpart = gpart + G, launch_pm_update checks), so each load's source
    // is a select of two bases, not a branch around each load
    const double *bp = a.gpart, *bk = a.cost + 2 - np;
    auto stage = [&](int base) {
        double v[SB];
#pragma unroll
        for (int u = 0; u < SB; u++) {
            const int j = min(base + u * PT, n - 1);
            v[u] = ld_sc1((j < np ? bp : bk) + j);
        }
#pragma unroll
        for (int u = 0; u < SB; u++) {
            const int j = base + u * PT;
            if (j < np) Lst[j] = v[u];
            else if (j < n) Lkey[j - np] = rank_key(v[u]);
        }
    };
    stage(t);   // the usual sizes: one batch, straight-line
    for (int base = t + PT * SB; base < n; base += PT * SB) stage(base);
    __syncthreads();
    stamp(6);
    if (s_last) {
        Status *st = a.status;
        const bool upd = !early && !wt, ok = !all_nan && !wt;
        // the normaliser (every thread, for its outputs and the status words) beside the first
        // output's gradient sum: two independent chains, each in block order
        double total = 0.0, g0 = 0.0;
        if (upd) sum2_in_order(Lst + G, 1, Lst + min(t, HC - 1), HC, nb, total, g0);
        // finish (mppi.cpp:421-447) and publish (178-182) of output o: gsum = sum_r e_r eps_r, uo = U*
        // as published, [lo, hi] its bounds
        auto finish = [&](int o, double gsum, double uo, double hi, double lo) {
            double u = Lus[o];
            if (upd) {
                const double gs = gsum / total;   // sum_r e_r eps_r / sum_r e_r
                a.gradient[o] = gs;
                u += gs * a.gradient_step;
                if (a.control_bound) u = smax(smin(u, hi), lo);
            }
            Lus[o] = u;
            if (upd || P.shift_by > 0) a.Us[o] = u;   // U*_shifted as sample() and the step leave it
            const double v = ok ? u : uo;
            if (ok) a.U[o] = v;
            pub(a.out + o, v);
        };
        if (t < HC) finish(t, g0, uo_t, hi_t, lo_t);
        for (int o = t + PT; o < HC; o += PT) {   // H C > PT: the rest, loaded here
            const int c = o % PC;
            finish(o, upd ? sum_in_order(Lst + o, nb, HC) : 0.0, a.U[o], a.control_bound ? a.cmax[c] : 0.0,
                   a.control_bound ? a.cmin[c] : 0.0);
        }
        if (t < a.X) a.x0_opt[t] = x0_t;
        if (t == 0) {
            st->all_nan = all_nan;
            st->early = early;
            st->minimum = mn;
            st->maximum = mx;
            if (upd) {
                st->total = total;
                st->tsplit[0] = total;
#pragma unroll
                for (int i = 1; i < GRAD_SPLIT; i++) st->tsplit[i] = 0.0;
            }
            st->sg_error = wt != 0;   // "the update threw": no filter() (as the finish kernels)
            pub(a.out + HC + 0, 0.0);      // (filter()'s cost is read behind the stream: wait_optimal)
            pub(a.out + HC + 1, (double)all_nan);
            pub(a.out + HC + 2, (double)early);
            pub(a.out + HC + 3, 0.0);
            pub(a.out + HC + 4, mn);
            pub(a.out + HC + 5, mx);
            pub(a.out + HC + 7, (double)wt);
        }
        if (t < CS_SLOTS) mppi_sample::reset_cost_stats(a.stats, t);   // every block has read them (ticket)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        stamp(7);
        if (t == 0) {
            st->wait_timeouts = 0;
            __hip_atomic_store(a.out + HC + 6, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        stamp(8);
    }
    // ---- tail: the next update's stable order and draws, behind the publish ----
    // rank (sample(), mppi.cpp:222-231) of the block's rollouts among rollouts 2..R-1 (keys staged
    // above): NaN last, ties by index; QD threads per rollout, each over its share of the keys
    {
        const int qd = t / PR;
        const int i = (int)g - 2;
        int cnt = 0;
        if (i >= 0 && i < S) {
            const uint64_t ki = Lkey[i];
            const int j0 = (S * qd) / QD, j1 = (S * (qd + 1)) / QD;
#pragma unroll 8
            for (int j = j0; j < j1; j++) {   // unrolled: the LDS reads of eight keys in flight
                const uint64_t kj = Lkey[j];
                cnt += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
            }
        }
        if (qd > 0) Lcnt[(qd - 1) * PR + rl] = cnt;
        __syncthreads();
        if (qd == 0 && i >= 0 && i < S) {
#pragma unroll
            for (int q = 1; q < QD; q++) cnt += Lcnt[(q - 1) * PR + rl];
            a.rank[g] = cnt;
        }
    }
    stamp(9);
    // the next update's draws (Philox by (rollout, step), its update index) into the buffer it will
    // sample from: rollouts >= 2 (rollout 0 is zero and rollout 1 -U* at sampling time)
    if (a.ahead_noise && row && g >= 2) {
        for (int k = t / PR; k < H; k += QD) {
            double e[PC];
            philox_eps(a, g, k, P.update_index + 1, e);
            double *o = a.ahead_noise + ((int64_t)k * a.Rpad + g) * PC;
#pragma unroll
            for (int c = 0; c < PC; c++) o[c] = e[c];
        }
    }
    if (fold && t == 0) *a.opt_cost = pm_rollout(a, LUf + HC, LUf, Lgm, nullptr, true);
    stamp(10);
}

namespace mppi_eng {

static size_t lds_bytes(int PR, int64_t R, int H)
{
    const int HC = H * PC;
    const int64_t nb = (R + PR - 1) / PR;
    return (size_t)((HC + H + 2 * PR + (R - 2) + pm_region(PR, HC, nb) + HC + 6) * 8 + (PT / PR - 1) * PR * 4);
}

// The in-launch grid barrier needs every block resident at once: the most blocks of each variant
// the device holds together (occupancy per CU at the variant's LDS, times the handle's CUs)
static int resident_blocks(int PR, size_t lds, unsigned cus, int lds_max)
{
    if (cus == 0 || lds > (size_t)lds_max) return 0;
    int per_cu = 0;
    hipError_t e = hipErrorInvalidValue;
    if (PR == 16) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pm_update_kernel<16>, PT, lds);
    else if (PR == 32) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pm_update_kernel<32>, PT, lds);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pm_update_kernel<64>, PT, lds);
    return e == hipSuccess ? per_cu * (int)cus : 0;
}

int pm_fused_rows(int64_t R, int H, unsigned cus, int lds_max)
{
    if (R < 4 || H < 1 || R > PM_FUSED_MAX_R) return 0;
    for (int PR = 16; PR <= 64; PR *= 2) {
        const int64_t nb = (R + PR - 1) / PR;
        const size_t lds = lds_bytes(PR, R, H);
        if (nb <= PM_FUSED_MAX_BLOCKS && lds <= 150 * 1024 && nb <= resident_blocks(PR, lds, cus, lds_max)) return PR;
    }
    return 0;
}

hipError_t launch_pm_update(const PmFusedArgs &a, hipStream_t s)
{
    // the handle's block count passed pm_fused_rows' residency check at create; each launch only
    // re-derives the rows per block from it (the occupancy queries behind pm_fused_rows, three per
    // launch, cost about a microsecond of every update's host path)
    int PR = 0;
    for (int p = 16; p <= 64 && !PR; p *= 2)
        if ((a.R + p - 1) / p == (int64_t)a.nblocks) PR = p;
    if (!PR || a.R < 4 || a.H < 1 || a.R > PM_FUSED_MAX_R || a.nblocks > PM_FUSED_MAX_BLOCKS)
        return hipErrorInvalidValue;   // the barrier and ticket targets assume the handle's count
    const unsigned nb = a.nblocks;
    if (a.tpart != a.gpart + (size_t)nb * a.H * PC) return hipErrorInvalidValue;   // the finisher's staging
    const size_t lds = lds_bytes(PR, a.R, a.H);
    if (lds > 150 * 1024) return hipErrorInvalidValue;
    if (PR == 16)
        hipLaunchKernelGGL(pm_update_kernel<16>, dim3(nb), dim3(PT), lds, s, a);
    else if (PR == 32)
        hipLaunchKernelGGL(pm_update_kernel<32>, dim3(nb), dim3(PT), lds, s, a);
    else
        hipLaunchKernelGGL(pm_update_kernel<64>, dim3(nb), dim3(PT), lds, s, a);
    return hipGetLastError();
}

}  // namespace mppi_eng
