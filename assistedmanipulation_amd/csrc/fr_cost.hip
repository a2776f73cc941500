// fr_cost.hip — the rollout costs of the cooperative FrankaRidgeback kernel, from its step records.
//
// fr_coop_kernel writes, for every (rollout, step k), the state x_k and the kinematics of the
// calculate() before it (kernels.hpp FR_NREC layout, rollout-major).  This kernel evaluates the
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

// Records of one rollout are contiguous ([R][H][FR_NREC]): a wave stages up to 64 of them into LDS
// with 1 KiB-contiguous loads, then each lane reads its step's record back.  The LDS record stride
// is 42 doubles (84 dwords), so the 16-byte reads of eight consecutive lanes hit distinct banks.
#ifdef COST_LDS_STAGE
constexpr int LREC2 = 21;   // LDS record stride in double2
#endif
constexpr int NREC2 = FR_NREC / 2;

#ifdef COST_LDS_STAGE
template <int CK, bool EN>
__global__ __launch_bounds__(64) void fr_step_cost_kernel(FrCostArgs a)
{
    __shared__ double2 L[64 * LREC2];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    const bool frow = a.fcost != nullptr && row == a.count;
    // no filter() when the update threw (mppi.cpp:170-176)
    if ((frow || a.optimal) && (a.status->all_nan || a.status->sg_error)) return;
    const int H = a.H;
    const double2 *rec = reinterpret_cast<const double2 *>(frow ? a.frec : a.rec + row * H * FR_NREC);
    const StepConst *stp = frow ? a.fsteps : a.steps;
    const DevCost &Cs = *a.cost;
    double J = 0.0;
    for (int base = 0; base < H; base += 64) {
        const int n = (H - base < 64) ? H - base : 64;
        const double2 *src = rec + (int64_t)base * NREC2;
        {   // all NREC2 loads in flight before the first LDS store
            double2 v[NREC2];
#pragma unroll
            for (int i = 0; i < NREC2; i++) {
                const int t = lane + 64 * i;
                v[i] = (t < n * NREC2) ? src[t] : double2{0.0, 0.0};
            }
#pragma unroll
            for (int i = 0; i < NREC2; i++) {
                const int t = lane + 64 * i, r = t / NREC2;
                L[r * LREC2 + (t - r * NREC2)] = v[i];
            }
        }
        __syncthreads();
        double c = 0.0;
        if (lane < n) {
            double r[FR_NREC];
#pragma unroll
            for (int i = 0; i < NREC2; i++) {
                const double2 v = L[lane * LREC2 + i];
                r[2 * i] = v.x;
                r[2 * i + 1] = v.y;
            }
            c = step_cost<CK, EN>(Cs, stp[base + lane], r, nullptr, nullptr);
        }
        for (int i = 0; i < n; i++) J += readlane_f64(c, i);
        __syncthreads();
    }
    if (lane != 0) return;
    J = isnan(J) ? (double)NAN : J;
    if (frow) *a.fcost = J;
    else if (a.optimal) *a.cost_out = J;
    else a.cost_out[a.begin + row] = J;
}
#else
// Lane k loads its step's record straight into registers (21 16-byte loads, 336 B apart across the
// lanes: every byte of the rollout's records is used once, through L2).  Staging through LDS took
// 21.5 KB per wave and held a CU to seven waves, too few to hide the loads; without it the kernel
// is bounded by registers (four waves per SIMD).
template <int CK, bool EN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void fr_step_cost_kernel(FrCostArgs a)
{
    __shared__ double Lj[FR_NB * JT_STRIDE];
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    const bool frow = a.fcost != nullptr && row == a.count;
    // no filter() when the update threw (mppi.cpp:170-176)
    if ((frow || a.optimal) && (a.status->all_nan || a.status->sg_error)) return;
    const int H = a.H;
    const double2 *rec = reinterpret_cast<const double2 *>(frow ? a.frec : a.rec + row * H * FR_NREC);
    const StepConst *stp = frow ? a.fsteps : a.steps;
    const DevCost &Cs = *a.cost;
    if (CK != CK_TRACK_POINT)   // per-joint parameters (84 of them for 64 lanes)
        for (int i = lane; i < FR_NB * JT_STRIDE; i += 64) {
            const int j = i / JT_STRIDE, f = i - j * JT_STRIDE;
            const double *src = f < 3 ? &Cs.lower[j].bound + f : (f < 6 ? &Cs.upper[j].bound + (f - 3) : &Cs.vel_q[j]);
            Lj[i] = *src;
        }
    __syncthreads();
    double J = 0.0;
    for (int base = 0; base < H; base += 64) {
        const int n = (H - base < 64) ? H - base : 64;
        const int k = base + (lane < n ? lane : 0);
        double r[FR_NREC];
        const double2 *src = rec + (int64_t)k * NREC2;
        constexpr int NLOAD = CK == CK_TRACK_POINT ? NREC2 : FR_NB;   // AssistedManipulation: the (q, qd) pairs
#pragma unroll
        for (int i = 0; i < NLOAD; i++) {
            const double2 v = src[i];
            r[2 * i] = v.x;
            r[2 * i + 1] = v.y;
        }
        const double c = step_cost<CK, EN>(Cs, stp[k], r, Lj, src);
        for (int i = 0; i < n; i++) J += readlane_f64(c, i);
    }
    if (lane != 0) return;
    J = isnan(J) ? (double)NAN : J;
    if (frow) *a.fcost = J;
    else if (a.optimal) *a.cost_out = J;
    else a.cost_out[a.begin + row] = J;
}
#endif

}  // namespace

namespace mppi_eng {

hipError_t launch_fr_step_cost(const FrCostArgs &a, hipStream_t s)
{
    const int64_t rows = a.count + (a.fcost ? 1 : 0);
    if (rows == 0) return hipSuccess;
    const dim3 grid((unsigned)rows), block(64);
    if (a.cost_kind == CK_TRACK_POINT) hipLaunchKernelGGL((fr_step_cost_kernel<CK_TRACK_POINT, false>), grid, block, 0, s, a);
    else if (a.energy) hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fr_step_cost_kernel<CK_ASSISTED_MANIPULATION, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace mppi_eng
