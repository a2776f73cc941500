// pm_fused.hip — one launch per point-mass update (BASELINE configs[1], 1024 x 32).
//
// The point-mass update (the a16 bring-up plugin: quadratic cost, ~25 flops per rollout-step) has
// no arithmetic to speak of; in five launches (sample, rollouts, weights + gradient, finish, rank)
// its time was the launches' fixed costs and their dependent memory trips.  Here one grid of
// 256-thread workgroups, each owning 64 rollouts, runs the whole of Trajectory::update
// (mppi.cpp:154-187) with one grid barrier:
//
//   phase A  sample (mppi.cpp:189-270): the block's eps columns into LDS (and the eps tensor):
//            rollout 0 zero, rollout 1 = -U*, kept rollouts the previous eps shifted, the rest
//            Philox by (rollout, step) - drawn ahead by the previous launch when it could; U*
//            shifted; then one wave rolls the 64 rollouts out of LDS (mppi.cpp:272-342) and folds
//            the costs' min / max / count into the CostStats slots (exact key atomics).
//   barrier  every block's costs and statistics are final.
//   phase B  optimise (mppi.cpp:344-418): e_r of the block's rollouts and its partial gradient
//            sum_r e_r eps_r over its 64 rollouts (fixed order), written through to L2 (sc1) for
//            the last block to arrive (agent-scope ticket), which adds the partials in block order,
//            steps U*, clamps and publishes the host block (mppi.cpp:421-447, 178-182), then runs
//            filter() (mppi.cpp:450-479) on one lane.
//   tail     while the host turns around: the stable rank of the block's rollouts (the next
//            update's keep-best) and the next update's Philox draws of its rollouts.
//
// Cross-block hand-offs follow MI355X_MICROARCH.md's measured forms: payloads stored sc1
// (write-through) and drained with vmcnt(0) before an agent-scope atomic add; readers poll with
// sc1 loads and load the payload with sc1 loads.  Every wait is bounded: a block that gives up
// counts it in Status::wait_timeouts, and the update then fails like the rollout launch's waits.
// A rollout's arithmetic is pm_rollout_kernel's (kernels.hip) operation for operation, so the
// costs are bit-identical to the five-launch path; the gradient and the normaliser are summed in
// another order (rounding only).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "sample_device.hpp"

using namespace mppi_eng;
using mppi_dev::smax;
using mppi_dev::smin;

namespace {

constexpr int PT = PM_FUSED_THREADS;   // threads per block
constexpr int PR = PM_FUSED_ROWS;      // rollouts per block (one wave rolls them out)
constexpr int PC = 3;                  // control dimension of the point mass
constexpr int BAR_SPINS = 1 << 22;     // about a second of s_sleep 1

__device__ __forceinline__ double ld_sc1(const double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// the rank's order (kernels.hip cost_key): order-preserving, -0 = +0, NaN last
__device__ __forceinline__ uint64_t rank_key(double c)
{
    return isnan(c) ? ~0ull : mppi_dev::cost_order_key(c);
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

// pm_rollout_kernel's horizon (kernels.hip pm_steps), the same operations in the same order; eps
// row k at eps[k * PC] (unused when optimal)
__device__ __forceinline__ double pm_rollout(const PmFusedArgs &a, const double *Lus, const double *Lgm, const double *eps,
                                             bool optimal)
{
    const DevPointMass &P = a.pm;
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = a.x0v[i];
    double J = 0.0;
#pragma unroll 4
    for (int k = 0; k < a.H; k++) {
        double u[3];
#pragma unroll
        for (int c = 0; c < 3; c++) u[c] = Lus[k * PC + c] + (optimal ? 0.0 : eps[k * PC + c]);
        double cost = 0.0;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const double d = x[i] - P.target[i];
            cost += P.q[i] * (d * d);
        }
#pragma unroll
        for (int i = 0; i < 3; i++) cost += P.r[i] * (u[i] * u[i]);
        const double sc = Lgm[k] * cost;
        if (!optimal && isnan(sc)) return NAN;   // rollout cost NaN, stop (mppi.cpp:331-334)
        J += sc;
#pragma unroll
        for (int i = 0; i < 3; i++) x[3 + i] = x[3 + i] + (u[i] * P.inv_mass) * a.dt;
#pragma unroll
        for (int i = 0; i < 3; i++) x[i] = x[i] + x[3 + i] * a.dt;
    }
    return J;
}

}  // namespace

// LDS (doubles): eps [PR][ES] (ES = H C + 1: the rollout wave's lanes then read distinct banks),
// U*_shifted [H C], gamma [H], the block's costs [PR] and e_r [PR], the rank's keys [R - 2] and
// partial counts [3][PR] (ints)
__global__ __launch_bounds__(PT) void pm_update_kernel(PmFusedArgs a)
{
    extern __shared__ double lds[];
    const int H = a.H, HC = H * PC, ES = HC + 1, t = threadIdx.x, w = t >> 6, l = t & 63;
    const int64_t S = a.R - 2;
    double *Leps = lds;
    double *Lus = Leps + PR * ES;
    double *Lgm = Lus + HC;
    double *Lcost = Lgm + H;
    double *Le = Lcost + PR;
    uint64_t *Lkey = reinterpret_cast<uint64_t *>(Le + PR);
    int *Lcnt = reinterpret_cast<int *>(Lkey + S);
    __shared__ int s_last;
    const int b = blockIdx.x, nb = gridDim.x;
    const int64_t r0 = (int64_t)b * PR;
    const SampleParams &P = a.sp;
    const double *Uprev = a.U;   // U* as the previous update published it
    const unsigned target = a.epoch * (unsigned)nb;
    auto stamp = [&](int i) {   // diagnostics: one clock stamp per block and phase
        if (a.stamps && t == 0) a.stamps[b * PM_STAMPS + i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // ---- phase A: sample (mppi.cpp:189-270) ----
    for (int i = t; i < HC; i += PT) {   // U*_shifted (mppi.cpp:197-207); unshifted, as last left
        const int k = i / PC, c = i - k * PC;
        Lus[i] = P.shift_by > 0 ? (k < P.shifted ? Uprev[(k + P.shift_by) * PC + c] : Uprev[(H - 1) * PC + c]) : a.Us[i];
    }
    for (int k = t; k < H; k += PT) Lgm[k] = a.steps[k].gamma_k;
    if (t == 0) s_last = 0;
    // the block's ranks once (LDS; Lcnt's room, used again only by the tail's rank)
    int *Lrank = Lcnt;
    if (t < PR) {
        const int64_t g = r0 + t;
        Lrank[t] = (g >= 2 && g < a.R) ? a.rank[g] : 0x7FFFFFFF;
    }
    __syncthreads();
    // items (step k, rollout): consecutive threads, consecutive rollouts; IB items per thread per pass
    // with their loads issued together (one memory trip per pass, not one per item)
    constexpr int IB = 4;
    for (int base = t; base < PR * H; base += PT * IB) {
        const double *src[IB];
        double sgn[IB], e[IB][PC];
        bool draw[IB], store[IB], live[IB];
        int kk[IB], rr[IB];
#pragma unroll
        for (int u = 0; u < IB; u++) {
            const int i = base + u * PT;
            const int k = i / PR, rl = i - k * PR;
            const int64_t g = r0 + rl;   // unsharded: local = global
            kk[u] = k;
            rr[u] = rl;
            live[u] = i < PR * H && g < a.R;
            src[u] = Uprev;   // any valid address
            sgn[u] = 1.0;
            draw[u] = false;
            store[u] = true;
            if (!live[u]) continue;
            const int rank = Lrank[rl];
            if (g == 0) {
                sgn[u] = 0.0;
            } else if (g == 1) {   // m_rollouts[1].noise = -m_optimal_control
                src[u] = Uprev + k * PC;
                sgn[u] = -1.0;
            } else if (rank < P.keep && (P.shift_by <= 0 || k < P.shifted)) {   // kept: the previous eps, shifted
                src[u] = a.prev + (((int64_t)k + (P.shift_by > 0 ? P.shift_by : 0)) * a.Rpad + g) * PC;
            } else if (a.ahead) {   // the previous launch's tail drew it into this update's buffer: in place
                src[u] = a.noise + ((int64_t)k * a.Rpad + g) * PC;
                store[u] = false;
            } else {
                draw[u] = true;
            }
        }
#pragma unroll
        for (int u = 0; u < IB; u++)
#pragma unroll
            for (int c = 0; c < PC; c++) e[u][c] = src[u][c];
#pragma unroll
        for (int u = 0; u < IB; u++) {
            const int i = base + u * PT;
            if (i >= PR * H) break;
            const int k = kk[u], rl = rr[u];
            if (!live[u]) {   // rows past R: zeros, which the gradient's fixed 64-row sum multiplies by 0
#pragma unroll
                for (int c = 0; c < PC; c++) Leps[rl * ES + k * PC + c] = 0.0;
                continue;
            }
            if (draw[u]) philox_eps(a, r0 + rl, k, P.update_index, e[u]);
            else if (sgn[u] != 1.0)
#pragma unroll
                for (int c = 0; c < PC; c++) e[u][c] = sgn[u] == 0.0 ? 0.0 : sgn[u] * e[u][c];   // rollout 0: +0
            double *o = a.noise + ((int64_t)k * a.Rpad + r0 + rl) * PC;
#pragma unroll
            for (int c = 0; c < PC; c++) {
                Leps[rl * ES + k * PC + c] = e[u][c];
                if (store[u]) o[c] = e[u][c];
            }
        }
    }
    if (b == 0 && t < a.X) a.x0_out[t] = a.x0v[t];
    __syncthreads();
    stamp(1);
    if (w == 0) {   // rollouts (mppi.cpp:272-342): one lane per rollout
        const int64_t g = r0 + l;
        double J = NAN;
        if (g < a.R) {
            J = pm_rollout(a, Lus, Lgm, Leps + l * ES, false);
            st_sc1(a.cost + g, J);   // read by every block's rank (tail)
        }
        Lcost[l] = J;
        // the block's min / max / count, then one exact key atomic each into CostStats slot b % 64
        const bool ok = g < a.R && !isnan(J);
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
        while (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && i < BAR_SPINS) {
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
            const int64_t g = r0 + l;
            const double c = Lcost[l];
            const double e = (g < a.R && !isnan(c)) ? exp(-a.cost_scale * (c - mn) / difference) : 0.0;
            Le[l] = e;
            if (g < a.R) a.wexp[g] = e;
            const double s = mppi_dev::wave_sum_dpp(e);
            if (l == 0) st_sc1(a.tpart + b, s);
        }
        __syncthreads();
        for (int o = t; o < HC; o += PT) {   // partial gradient: the block's rollouts in order
            double acc = 0.0;
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
    if (s_last) {
        Status *st = a.status;
        const int wt = __hip_atomic_load(&st->wait_timeouts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool upd = !early && !wt, ok = !all_nan && !wt;
        double total = 0.0;
        if (upd)
            for (int i = 0; i < nb; i++) total += ld_sc1(a.tpart + i);
        for (int o = t; o < HC; o += PT) {   // finish (mppi.cpp:421-447) and publish (178-182)
            const int c = o % PC;
            double u = Lus[o];
            if (upd) {
                double g = 0.0;
                for (int i = 0; i < nb; i++) g += ld_sc1(a.gpart + (int64_t)i * HC + o);
                g /= total;   // sum_r e_r eps_r / sum_r e_r
                a.gradient[o] = g;
                u += g * a.gradient_step;
                if (a.control_bound) u = smax(smin(u, a.cmax[c]), a.cmin[c]);
            }
            Lus[o] = u;
            if (upd || P.shift_by > 0) a.Us[o] = u;   // U*_shifted as sample() and the step leave it
            const double v = ok ? u : a.U[o];
            if (ok) a.U[o] = v;
            a.out[o] = v;
        }
        if (t < a.X) a.x0_opt[t] = a.x0v[t];
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
            a.out[HC + 0] = *a.opt_cost;
            a.out[HC + 1] = (double)all_nan;
            a.out[HC + 2] = (double)early;
            a.out[HC + 3] = 0.0;
            a.out[HC + 4] = mn;
            a.out[HC + 5] = mx;
            a.out[HC + 7] = (double)wt;
        }
        if (t < CS_SLOTS) mppi_sample::reset_cost_stats(a.stats, t);   // every block has read them (ticket)
        __syncthreads();
        if (t == 0) {
            st->wait_timeouts = 0;
            __threadfence_system();
            __hip_atomic_store(a.out + HC + 6, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            stamp(5);
            // filter() (mppi.cpp:450-479): the cost of the published U* from this update's state,
            // while the host takes the result; none when the update threw
            if (ok) *a.opt_cost = pm_rollout(a, Lus, Lgm, nullptr, true);
        }
    }
    // ---- tail: the next update's stable order and draws, behind the publish ----
    // rank (sample(), mppi.cpp:222-231) of the block's rollouts among rollouts 2..R-1: NaN last,
    // ties by index; four threads per rollout, each over a quarter of the keys (staged in LDS from
    // sc1 loads: the other blocks stored them this launch)
    for (int64_t j = t; j < S; j += PT) Lkey[j] = rank_key(ld_sc1(a.cost + 2 + j));
    __syncthreads();
    {
        const int rl = t & (PR - 1), qd = t >> 6;
        const int64_t i = r0 + rl - 2;
        int cnt = 0;
        if (i >= 0 && i < S) {
            const uint64_t ki = Lkey[i];
            const int64_t j0 = (S * qd) / 4, j1 = (S * (qd + 1)) / 4;
#pragma unroll 8
            for (int64_t j = j0; j < j1; j++) {   // unrolled: the LDS reads of eight keys in flight
                const uint64_t kj = Lkey[j];
                cnt += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
            }
        }
        if (qd > 0) Lcnt[(qd - 1) * PR + rl] = cnt;
        __syncthreads();
        if (qd == 0 && i >= 0 && i < S) a.rank[i + 2] = cnt + Lcnt[rl] + Lcnt[PR + rl] + Lcnt[2 * PR + rl];
    }
    stamp(6);
    // the next update's draws (Philox by (rollout, step), its update index) into the buffer it will
    // sample from: rollouts >= 2 (rollout 0 is zero and rollout 1 -U* at sampling time)
    if (a.ahead_noise) {
        for (int i = t; i < PR * H; i += PT) {
            const int k = i / PR, rl = i - k * PR;
            const int64_t g = r0 + rl;
            if (g < 2 || g >= a.R) continue;
            double e[PC];
            philox_eps(a, g, k, P.update_index + 1, e);
            double *o = a.ahead_noise + ((int64_t)k * a.Rpad + g) * PC;
#pragma unroll
            for (int c = 0; c < PC; c++) o[c] = e[c];
        }
    }
    stamp(7);
}

namespace mppi_eng {

size_t pm_fused_lds_bytes(int64_t R, int H)
{
    const int64_t HC = (int64_t)H * PC;
    return (size_t)((PR * (HC + 1) + HC + H + 2 * PR + (R - 2)) * 8 + 3 * PR * 4);
}

bool pm_fused_fits(int64_t R, int H)
{
    return R >= 4 && H >= 1 && R <= PM_FUSED_MAX_R && (int64_t)H * PC <= 4 * PT && pm_fused_lds_bytes(R, H) <= 150 * 1024;
}

hipError_t launch_pm_update(const PmFusedArgs &a, hipStream_t s)
{
    if (!pm_fused_fits(a.R, a.H)) return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((a.R + PR - 1) / PR);
    if (nb != a.nblocks) return hipErrorInvalidValue;   // the barrier and ticket targets assume it
    hipLaunchKernelGGL(pm_update_kernel, dim3(nb), dim3(PT), pm_fused_lds_bytes(a.R, a.H), s, a);
    return hipGetLastError();
}

}  // namespace mppi_eng
