// fr_cost.hip — the rollout costs of the cooperative FrankaRidgeback kernel, from its step records.
//
// fr_coop_kernel writes, for every (rollout, step k), the state x_k and the kinematics of the
// calculate() before it (kernels.hpp FR_REC layout, rollout-major).  This kernel evaluates the
// objective on all of them at once: one wave per rollout, one lane per step, so every lane does distinct work
// (inside the rollout kernel the workspace, trajectory and manipulability terms are row-uniform
// and all 16 lanes of a row would repeat them).  The step costs are then summed in step order,
// J = ((c_0 + c_1) + c_2) + ..., as the reference accumulates them (mppi.cpp:322-337).
//
// NaN: the reference stops a rollout at its first NaN step cost and sets J = NaN; a NaN step cost
// makes this sum NaN as well, and the steps after it do not matter.  The sum is canonicalised to
// the quiet NaN the reference stores.
//
// AssistedManipulation::get_cost (assisted_manipulation.cpp:58-128) and TrackPoint::get_cost
// (frankaridgeback/objective/track_point.cpp:10-34), term order kept.  The joint-limit and
// velocity sums keep the association of the lane sums they replace: (joints 0..5) + (6..11).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "device_common.hpp"
#include "engine_types.hpp"
#include "kernels.hpp"
#include "fr_cost_terms.hpp"

using namespace mppi_eng;
using mppi_dev::smin;

namespace {

using namespace mppi_cost;

// Lane k loads its step's record straight into registers (21 16-byte loads, 336 B apart across the
// lanes: every byte of the rollout's records is used once, through L2).  Staging through LDS took
// 21.5 KB per wave and held a CU to seven waves, too few to hide the loads; without it the kernel
// is bounded by registers (four waves per SIMD).
template <int CK, bool EN, bool KC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void fr_step_cost_kernel(FrCostArgs a)
{
    __shared__ double Lj[FR_NB * JT_STRIDE];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    const bool frow = a.fcost != nullptr && row == a.count;
    // no filter() when the update threw (mppi.cpp:170-176)
    if ((frow || a.optimal) && (a.status->all_nan || a.status->sg_error)) return;
    const int H = a.H;
    const StepConst *stp = frow ? a.fsteps : a.steps;
    const DevCost &Cs = *a.cost;
    if (CK != CK_TRACK_POINT)   // per-joint parameters (84 of them for 64 lanes)
        for (int i = lane; i < FR_NB * JT_STRIDE; i += 64) {
            const int j = i / JT_STRIDE, f = i - j * JT_STRIDE;
            const double *src = f < 3 ? &Cs.lower[j].bound + f : (f < 6 ? &Cs.upper[j].bound + (f - 3) : &Cs.vel_q[j]);
            Lj[i] = *src;
        }
    __syncthreads();
    const double J = rollout_cost<CK, EN, JT_STRIDE, KC>(Cs, stp, frow ? a.frec : a.rec + row * H * (KC ? FR_REC_C : FR_REC), H,
                                                         lane, Lj);
    if (lane != 0) return;
    if (frow) *a.fcost = J;
    else if (a.optimal) *a.cost_out = J;
    else {
        a.cost_out[a.begin + row] = J;
        fold_cost_stats(a.stats, J, row);   // exact min / max / count, any order
    }
}

// The optimal rollout's per-term totals (AssistedManipulation's accumulators after filter(),
// mppi.cpp:450-479 with thread 0's cost, reset at its start): one wave over the filter() row's
// records, lane = step, each term summed over the steps in step order (m_*_cost += per step).
__global__ __launch_bounds__(64) void fr_terms_kernel(const DevCost *cost, const StepConst *steps, const double *rec, int H,
                                                      int compact, double *out7)
{
    const int lane = threadIdx.x;
    double tot[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int base = 0; base < H; base += 64) {
        const int n = (H - base < 64) ? H - base : 64;
        const int k = base + (lane < n ? lane : 0);
        double t[7], r[FR_NREC];
        derive_record(rec + (int64_t)k * (compact ? FR_REC_C : FR_REC), r, compact != 0);
        assisted_manipulation_terms(*cost, steps[k], r, r[REC_QQD + 4], t);
#pragma unroll
        for (int m = 0; m < 7; m++)
            for (int i = 0; i < n; i++) tot[m] += readlane_f64(t[m], i);
    }
    if (lane < 7) {
        double v = tot[0];
#pragma unroll
        for (int m = 1; m < 7; m++) v = lane == m ? tot[m] : v;
        out7[lane] = v;
    }
}

}  // namespace

namespace mppi_eng {

hipError_t launch_fr_terms(const DevCost *cost, const StepConst *steps, const double *rec, int H, bool compact, double *out7,
                           hipStream_t s)
{
    hipLaunchKernelGGL(fr_terms_kernel, dim3(1), dim3(64), 0, s, cost, steps, rec, H, compact ? 1 : 0, out7);
    return hipGetLastError();
}

hipError_t launch_fr_step_cost(const FrCostArgs &a, hipStream_t s)
{
    const int64_t rows = a.count + (a.fcost ? 1 : 0);
    if (rows == 0) return hipSuccess;
    const dim3 grid((unsigned)rows), block(64);
    // the records' layout is the launch's that wrote them (FrCostArgs::compact)
    if (a.compact) {
        if (a.cost_kind == CK_TRACK_POINT) hipLaunchKernelGGL((fr_step_cost_kernel<CK_TRACK_POINT, false, true>), grid, block, 0, s, a);
        else if (a.energy) hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, true, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, false, true>), grid, block, 0, s, a);
    } else {
        if (a.cost_kind == CK_TRACK_POINT) hipLaunchKernelGGL((fr_step_cost_kernel<CK_TRACK_POINT, false, false>), grid, block, 0, s, a);
        else if (a.energy) hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, true, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, false, false>), grid, block, 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace mppi_eng
