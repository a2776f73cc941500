// engine.cpp — host runtime of the MI355X MPPI engine: the C-ABI of include/mppi_amd.h.
//
// Replaces mppi::Trajectory (reference src/controller/mppi.{hpp,cpp}).  The host keeps the
// reference's scalar bookkeeping (shift count, times, counters, the published U* for get());
// every per-rollout array lives in HBM and is produced by the kernels of kernels.hip.
// One handle = one HIP device + one stream (+ one RCCL communicator when sharded).

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

// Host arithmetic mirrors the reference's double expressions exactly (shift counts, step
// constants): no FMA contraction.
#pragma clang fp contract(off)

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mppi_amd.h"
#include "../../include/mppi_amd_frankaridgeback.h"
#include "engine_types.hpp"
#include "kernels.hpp"

using namespace mppi_eng;

namespace mppi_eng {
EnvSwitches env_switches_read()
{
    auto is = [](const char *name, char c) { const char *e = std::getenv(name); return e && e[0] == c; };
    EnvSwitches e{};
    e.draw_ahead_off = is("MPPI_DRAW_AHEAD", '0');
    e.tail_draws_off = is("MPPI_TAIL_DRAWS", '0');
    e.pm_fused_off = is("MPPI_PM_FUSED", '0');
    e.costs_in_launch_off = is("MPPI_COSTS_IN_LAUNCH", '0');
    e.handover_off = is("MPPI_HANDOVER", '0');
    e.split_off = is("MPPI_SPLIT", '0');
    e.stream_prio_off = is("MPPI_STREAM_PRIO", '0');
    const char *rk = std::getenv("MPPI_RELAY_K");
    e.relay_k = (rk && rk[0] >= '1' && rk[0] <= '0' + RELAY_K_MAX) ? rk[0] - '0' : 0;
    return e;
}
}  // namespace mppi_eng

namespace {

std::string g_last_error;

struct DeviceBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct mppi_handle {
    int device = 0;
    EnvSwitches env{};   // the A/B switches as the environment held them at create (env_switches_read)
    hipStream_t stream = nullptr;
    hipStream_t stream_opt = nullptr;   // filter(): optimal rollout, overlapped with the next update

    hipEvent_t ev[6] = {};
    hipEvent_t ev_pub = nullptr, ev_opt_done = nullptr, ev_opt_end = nullptr;
    hipEvent_t ev_dyn = nullptr;   // after the rollout (dynamics) kernel, before the cost kernel
    hipEvent_t ev_wg = nullptr;    // timing level 2: after weights_gradient_kernel (kernel_ms[6])
    hipEvent_t ev_ar = nullptr;    // timing level 2, RCCL-sharded: after the cost all-reduce (kernel_ms[7])
    // filter() (the optimal rollout) of the last update: pending (not launched yet: it rides in the
    // next update's remainder launch, or runs alone when something needs it first), launched
    enum { OPT_NONE, OPT_PENDING, OPT_LAUNCHED, OPT_FOLDED } opt_state = OPT_NONE;
    const StepConst *opt_steps = nullptr;   // the step constants its update used
    // sample, rollout (dynamics + cost kernels), reduce, optimal rollout, update, dynamics kernel,
    // the weight reduce alone, the cost all-reduce (RCCL-sharded)
    float kernel_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // HIP-event timing on the update path (mppi_set_timing): 0 none, 1 the rollout kernel alone
    // ([5]), 2 every phase.  Each event record costs the stream a few microseconds between kernels.
    int timing = 0;
    // timing level 1 records the rollout launch's event pair into a ring; the elapsed times are
    // read later (mppi_rollout_kernel_times), not in the update that recorded them: reading one
    // right behind the publish held the host ~70 us before it returned
    static constexpr int EV_RING = 64;
    hipEvent_t ev_ring[2 * EV_RING] = {};
    int ring_head = 0, ring_count = 0;   // next pair to record; recorded pairs not yet read
    bool ring_unread = false;            // kernel_ms[5] not yet taken from the newest pair
    // the update's rollout launch drew the next update's eps for its main waves' rows (tail_draws):
    // phase 3 draws only the rows it left (launch_draw_ahead's subset)
    bool tail_drawn = false;
    // what the last update's rollout launch did (mppi_update_info)
    int64_t info[MPPI_UPDATE_INFO_N] = {};
    int tail_nxb = 0;
    int64_t tail_xbase = 0, tail_row0 = 0;
    // MPPI_HOST_TRACE=1: host-side turnaround stamps, averaged and printed by mppi_destroy:
    // [0] flag seen -> phase 3 returns, [1] return -> next phase 1, [2] phase 1 -> rollout launched
    bool host_trace = false;
    std::chrono::steady_clock::time_point ht_flag, ht_ret;
    double ht_sum[3] = {0, 0, 0};
    int64_t ht_n[3] = {0, 0, 0};
    int dyn_kind = 0, cost_kind = 0;
    int64_t S = 0, K = 0, R = 0, H = 0, C = 0, X = 0;
    double dt = 0, gradient_step = 0, cost_scale = 0, gamma = 1;
    int control_bound = 0;
    std::vector<double> cmin, cmax, cdefault, init_state, T;
    bool has_default = false, tdiag = false;
    int sg_window = 0, sg_order = 0;
    // sharding
    int world = 1, rank = 0;
    int64_t begin = 0, count = 0, Rpad = 0;
    ncclComm_t comm = nullptr;
    bool updated_once = false;
    // reference scalar state (mppi.hpp:545-657)
    double last_shift_time = 0, rollout_time = 0, last_rollout_time = 0, update_last = 0, update_duration = 0;
    uint64_t update_count = 0;
    // the publish flag's sequence: one per phase-3 call, success or failure (update_count only
    // counts successes, so a failed update must not leave the flag at the next update's value)
    uint64_t publish_seq = 0;
    // draws ahead (launch_draw_ahead behind phase 3): valid for the update whose inputs match
    struct AheadSig {
        uint64_t update_index, seed;
        int64_t begin, count, H, C;
    } ahead{};
    bool ahead_valid = false;
    int64_t shift_by = 0, shifted = 0;
    int compat_uint8 = 0;
    double publish_timeout_s = 5.0;   // floor of the bounded publish wait (phase 3)
    int noise_source = MPPI_NOISE_DEVICE_PHILOX;
    uint64_t seed = 0x5EEDull;
    std::vector<double> inj_pending;
    // published (host) — guarded by mtx for get() concurrent with update()
    std::mutex mtx;
    std::vector<double> U_host;
    double opt_cost = 0;
    // forecast / per-step constants
    std::vector<double> forecast;   // H x 6 caller table (mppi_set_forecast)
    struct DeviceForecast {         // mppi_forecast_attach (forecast.hip)
        int type = FC_NONE;
        double horison = 0, valid_until = 0, value[6] = {0, 0, 0, 0, 0, 0};   // LOCF / Average mean
        double window = 0, last = 0;                                          // Average
        std::vector<std::pair<double, std::array<double, 6>>> buffer;
        int order = 0, n = 0, steps = 0;                                      // Kalman
        double time_step = 0, last_update = 0;
        int64_t pending = 0;
        DevKalman *d_kf = nullptr;
        double *d_pred = nullptr;
    } fc;
    double *d_gamma = nullptr;      // [H] pow(gamma, k) (host std::pow)
    double *d_fc_out = nullptr;     // [6] forecast_eval result
    double *d_terms = nullptr;      // [7] mppi_optimal_terms
    StepConst *d_steps_buf[2] = {nullptr, nullptr};   // per-update constants, alternate updates
    mppi_assisted_manipulation_desc am{};
    mppi_quadratic_cost_desc quad{};
    double pm_mass = 1.0;
    // device buffers
    DevModel *d_model = nullptr;
    DevCost *d_cost = nullptr;
    double *d_table = nullptr;   // cooperative kernels' body table (built from d_model, d_cost)
    DevPointMass *d_pm = nullptr;
    StepConst *d_steps = nullptr;
    double *d_x0 = nullptr, *d_U = nullptr, *d_Us = nullptr, *d_noise = nullptr, *d_noise_prev = nullptr, *d_costs = nullptr;
    double *d_gpart = nullptr, *d_grad = nullptr, *d_T = nullptr, *d_inj = nullptr, *d_opt = nullptr;
    double *d_cmin = nullptr, *d_cmax = nullptr, *d_x0_opt = nullptr, *d_gsplit = nullptr;
    CostStats *d_cstats = nullptr;
    // sharded with an engine-owned communicator: the rank's costs at their global slots, zero
    // elsewhere for good (nothing writes those), all-reduced out of place into d_costs - no clear
    // per update (a fill launch and its gap)
    double *d_costs_local = nullptr;   // the update's cost min / max / count (cost kernel atomics)
    double *d_wexp = nullptr, *d_wpart = nullptr;   // unnormalised weights e_r; large-R softmin partials
    // cooperative kernel's step records [Rpad][H][FR_REC] and the filter() row's [H][FR_REC]
    double *d_rec = nullptr, *d_rec_opt = nullptr;
    RelayXfer *d_rx = nullptr;     // the relay's hand-offs between workgroups (fr_coop.hip relay_stage)
    uint32_t relay_token = 0;      // one per rollout launch (nonzero)
    bool opt_rec_compact = false;   // d_rec_opt holds compact records (the standalone filter()), else 768-B ones (folded)
    uint32_t *d_trace = nullptr;   // MPPI_WAVE_TRACE=<file>: per-block timing of the rollout kernel (COOP_TRACE builds)
    std::string trace_path;
    size_t inj_capacity = 0;   // doubles
    int *d_rank = nullptr;
    uint64_t *d_rank_keys = nullptr;   // rank scratch: chunk-sorted cost keys
    Status *d_status = nullptr;
    double *d_sg_w = nullptr, *d_sg_uu = nullptr, *d_sg_tt = nullptr, *d_sg_last = nullptr;
    int64_t *d_sg_start = nullptr;
    double *h_out = nullptr;     // pinned [HC + 8], mapped: finish_kernel writes it over the bus
    double *h_out_dev = nullptr; // its device address
    double *h_opt = nullptr;     // pinned: optimal cost copied back on the side stream
    std::vector<void *> allocations;
    std::string err;
    // hipGraph path (mppi_set_graph / MPPI_GRAPH=1): the steady-state update's launches (rollout,
    // weights + gradient, finish, rank + draws ahead; sharded, the two RCCL all-reduces between
    // them) captured once and replayed with each update's arguments written into the executable
    // graph's kernel nodes
    int graph_mode = 0;
    bool graph_dry = false;             // phases fill `gargs` instead of launching
    struct GraphArgs {
        FrRolloutArgs roll, roll2;   // the rollout launch (the split's two: roll, roll2)
        int nroll = 1;
        WGradArgs wg;
        FinishArgs fin;
        RankDrawLaunch rd;
        bool x_kernel = false, folded = false;
    } gargs;
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    struct GraphNode {
        hipGraphNode_t node;
        int kind;   // GraphKernel; GK_ROLLOUT nodes in capture order: the split's first, then its second
        int index;  // the kind's node count before this one
        hipKernelNodeParams params;
    };
    std::vector<GraphNode> gnodes;   // the kernel nodes whose arguments each update rewrites
    int64_t graph_updates = 0;          // updates that ran as the graph (diagnostics)
    int64_t graph_failures = 0;         // captures that failed (the update then ran eagerly)
    std::string graph_error;            // why the last one failed
    int debug_graph_fail = 0;           // mppi_debug_inject(MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL, n)
    // in-launch waits that gave up (fr_coop.hip note_wait_timeout), summed over the updates
    int64_t wait_timeouts_total = 0;
    // mppi_debug_inject: fault bits for the next debug_updates rollout launches (tests only)
    int debug_flags = 0, debug_updates = 0;
    bool published_once = false;   // an update has published U* (and so has a filter() row)
    // the point mass in one launch per update (pm_fused.hip, launch_pm_update)
    DevPointMass pm_host{};
    unsigned *d_pm_sync = nullptr;   // [2] grid-barrier and ticket counters (monotonic)
    double *d_pm_part = nullptr;     // [nblocks][H C] partial gradients, then [nblocks] normalisers
    unsigned pm_epoch = 0, pm_nblocks = 0;
    uint64_t *d_pm_stamps = nullptr;   // MPPI_PM_STAMPS=1: the launch's phase stamps per block
    std::vector<double> pm_stamp_sum; // their per-phase sums (us after the block's entry), printed at destroy
    int64_t pm_stamp_n = 0;
    // per-update phase state
    bool phase_open = false;
    std::chrono::steady_clock::time_point t_start;
    double phase_time = 0;
};

static mppi_status launch_filter_standalone(mppi_handle *h);

namespace {

mppi_status fail(mppi_handle *h, mppi_status st, const std::string &msg)
{
    if (h) h->err = msg;
    else g_last_error = msg;
    return st;
}

#define HIP_TRY(expr)                                                                                          \
    do {                                                                                                       \
        hipError_t e_ = (expr);                                                                                \
        if (e_ != hipSuccess) return fail(h, MPPI_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

#define NCCL_TRY(expr)                                                                                              \
    do {                                                                                                            \
        ncclResult_t r_ = (expr);                                                                                   \
        if (r_ != ncclSuccess) return fail(h, MPPI_ERR_COMM, std::string(#expr ": ") + ncclGetErrorString(r_));    \
    } while (0)

template <class T>
hipError_t dalloc(mppi_handle *h, T **p, size_t n)
{
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    h->allocations.push_back(q);
    *p = (T *)q;
    return hipMemset(q, 0, std::max<size_t>(n, 1) * sizeof(T));
}

// Gaussian::set_covariance (gaussian.hpp:48-55): T = V sqrt(L); any T with T T^T = Sigma gives
// the same distribution (parity runs inject eps).  Diagonal Sigma -> T = diag(sqrt).
void noise_transform(int n, const double *cov_colmajor, std::vector<double> &T, bool &diag)
{
    diag = true;
    for (int c = 0; c < n; c++)
        for (int r = 0; r < n; r++)
            if (r != c && cov_colmajor[(size_t)c * n + r] != 0.0) diag = false;
    T.assign((size_t)n * n, 0.0);
    if (diag) {
        for (int i = 0; i < n; i++) T[(size_t)i * n + i] = std::sqrt(std::max(0.0, cov_colmajor[(size_t)i * n + i]));
        return;
    }
    std::vector<double> A((size_t)n * n), V((size_t)n * n, 0.0);
    for (int c = 0; c < n; c++)
        for (int r = 0; r < n; r++) A[(size_t)r * n + c] = 0.5 * (cov_colmajor[(size_t)c * n + r] + cov_colmajor[(size_t)r * n + c]);
    for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {   // cyclic Jacobi
        double off = 0;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) off += A[(size_t)p * n + q] * A[(size_t)p * n + q];
        if (off < 1e-30) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[(size_t)p * n + q];
                if (std::fabs(apq) < 1e-300) continue;
                const double theta = (A[(size_t)q * n + q] - A[(size_t)p * n + p]) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                const double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; k++) {
                    const double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
                    A[(size_t)k * n + p] = c * akp - s * akq;
                    A[(size_t)k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    const double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
                    A[(size_t)p * n + k] = c * apk - s * aqk;
                    A[(size_t)q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    const double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
                    V[(size_t)k * n + p] = c * vkp - s * vkq;
                    V[(size_t)k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int j = 0; j < n; j++) {
        const double l = std::sqrt(std::max(0.0, A[(size_t)j * n + j]));
        for (int i = 0; i < n; i++) T[(size_t)i * n + j] = V[(size_t)i * n + j] * l;
    }
}

// --- Savitzky-Golay weights (gram_savitzky_golay.cpp: GramPoly / GenFact / Weight) ----------
double gram_poly(int i, int m, int k, int s)
{
    if (k > 0)
        return (4. * k - 2.) / (k * (2. * m - k + 1.)) * (i * gram_poly(i, m, k - 1, s) + s * gram_poly(i, m, k - 1, s - 1)) -
               ((k - 1.) * (2. * m + k)) / (k * (2. * m - k + 1.)) * gram_poly(i, m, k - 2, s);
    return (k == 0 && s == 0) ? 1. : 0.;
}
double gen_fact(int a, int b)
{
    double gf = 1.;
    for (int j = (a - b) + 1; j <= a; j++) gf *= j;
    return gf;
}
std::vector<double> sg_weights(int m, int n)
{
    std::vector<double> w(2 * (size_t)m + 1);
    for (int i = 0; i < 2 * m + 1; ++i) {
        double v = 0;
        for (int k = 0; k <= n; ++k)
            v = v + (2 * k + 1) * (gen_fact(2 * m, k) / gen_fact(2 * m + k + 1, k + 1)) * gram_poly(i - m, m, k, 0) * gram_poly(0, m, k, 0);
        w[(size_t)i] = v;
    }
    return w;
}

double left_barrier_h(const mppi_barrier &b, double v)
{
    if (v <= b.bound) {
        const double d = b.bound - v;
        return b.maximum_cost + b.scale * (d * d);
    }
    const double x = b.scale / (v - b.bound);
    return (b.maximum_cost < x) ? b.maximum_cost : x;
}

DevBarrier devb(const mppi_barrier &b) { return DevBarrier{b.bound, b.scale, b.maximum_cost}; }

// trajectory_cost()'s constants for the wrench F (force part) (assisted_manipulation.cpp:237-290)
StepConst step_const(const mppi_assisted_manipulation_desc &a, const double *F, bool have_forecast, double gamma_k)
{
    StepConst s{};
    s.gamma_k = gamma_k;
    const double mx = a.trajectory_target_maximum;
    for (int i = 0; i < 3; i++) {
        double t = a.trajectory_target_scale * F[i];
        t = (mx < t) ? mx : t;           // cwiseMin(max)
        t = (t < -mx) ? -mx : t;         // cwiseMax(-max)
        s.target[i] = t;
    }
    s.tt = (s.target[0] * s.target[0] + s.target[1] * s.target[1]) + s.target[2] * s.target[2];
    const double distance = std::sqrt(s.tt);
    s.active = (have_forecast && a.has_forecast && distance > a.trajectory_position_threshold) ? 1 : 0;
    const mppi_quadratic &pc = a.trajectory_position_cost;
    s.pos_cost = (pc.constant_cost + pc.linear_cost * std::fabs(distance)) + pc.quadratic_cost * distance * distance;
    double vt = std::exp(a.trajectory_velocity_dropoff * distance) - 1;
    vt = (vt < a.trajectory_velocity_minimum) ? a.trajectory_velocity_minimum : ((a.trajectory_velocity_maximum < vt) ? a.trajectory_velocity_maximum : vt);
    s.vtarget = vt;
    return s;
}

// trajectory_cost() per-step constants and pow(gamma, k) (mppi.cpp:326).
void build_steps(const mppi_handle *h, std::vector<StepConst> &steps)
{
    steps.assign((size_t)h->H, StepConst{});
    for (int64_t k = 0; k < h->H; k++) {
        const double gk = std::pow(h->gamma, (double)k);
        if (h->cost_kind != MPPI_COST_ASSISTED_MANIPULATION) {
            steps[(size_t)k].gamma_k = gk;
            continue;
        }
        double F[3] = {0, 0, 0};
        if (!h->forecast.empty())
            for (int i = 0; i < 3; i++) F[i] = h->forecast[(size_t)(6 * k + i)];
        steps[(size_t)k] = step_const(h->am, F, true, gk);
    }
}

mppi_status upload_steps(mppi_handle *h)
{
    std::vector<StepConst> steps;
    build_steps(h, steps);
    for (StepConst *d : h->d_steps_buf)
        HIP_TRY(hipMemcpyAsync(d, steps.data(), steps.size() * sizeof(StepConst), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MPPI_OK;
}

// The objective's device block (DevCost) from its descriptor: AssistedManipulation's
// configuration, or TrackPoint's, with the self-collision constant of the zero link positions.
void build_dev_cost(const mppi_cost_desc &cost, DevCost &c)
{
    const mppi_assisted_manipulation_desc &a = cost.assisted_manipulation;
    c.kind = cost.kind;
    // the 20 link pairs of both objectives' self_collision_cost (Link enum: PIVOT = 3,
    // PANDA_LINK1..7 = 4..10; radii index = link - 3), link positions the zero stub
    static const int pairs[20][2] = {{3, 6}, {3, 7}, {3, 8}, {3, 9}, {3, 10}, {4, 6}, {4, 7}, {4, 8}, {4, 9}, {4, 10},
                                     {5, 7}, {5, 8}, {5, 9}, {5, 10}, {6, 8}, {6, 9}, {6, 10}, {7, 9}, {7, 10}, {8, 10}};
    if (cost.kind == MPPI_COST_TRACK_POINT) {
        const mppi_track_point_desc &t = cost.track_point;
        c.tp_en_joint = t.enable_joint_limits;
        c.tp_en_self = t.enable_self_collision_avoidance;
        c.tp_en_reach = t.enable_reach_limits;
        for (int i = 0; i < 3; i++) c.tp_point[i] = t.point[i];
        // joint_limit_cost's static limits (track_point.cpp:45-66)
        static const double lo[FR_NB] = {-2.0, -2.0, -6.28, -2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973, 0.5, 0.5};
        static const double up[FR_NB] = {2.0, 2.0, 6.28, 2.8973, 1.7628, 2.8973, 0.0698, 2.8973, 3.7525, 2.8973, 0.5, 0.5};
        for (int i = 0; i < FR_NB; i++) {
            c.tp_lo[i] = lo[i];
            c.tp_up[i] = up[i];
        }
        double sc = 0.0;   // track_point.cpp:97-160: collision = radii - distance
        for (auto &p : pairs) {
            const double distance = std::sqrt((0.0 * 0.0 + 0.0 * 0.0) + 0.0 * 0.0);
            const double radii = t.self_collision_radii[p[0] - 3] + t.self_collision_radii[p[1] - 3];
            sc += left_barrier_h(t.self_collision_limit, radii - distance);
        }
        c.tp_self = sc;
        c.tp_reach = devb(t.maximum_reach_limit);
    } else {
        c.en_joint = a.enable_joint_limit;
        c.en_self = a.enable_self_collision_limit;
        c.en_work = a.enable_workspace_limit;
        c.en_energy = a.enable_energy_limit;
        c.en_below = devb(a.energy_limit_below);
        c.en_above = devb(a.energy_limit_above);
        c.en_vel = a.enable_velocity_cost;
        c.en_traj = a.enable_trajectory_cost;
        c.en_manip = a.enable_manipulability_cost;
        for (int i = 0; i < FR_NB; i++) {
            c.lower[i] = devb(a.lower_joint_limit[i]);
            c.upper[i] = devb(a.upper_joint_limit[i]);
            c.vel_q[i] = a.velocity_cost[i].quadratic_cost;
        }
        // self_collision_cost with get_link_position == 0 (assisted_manipulation.cpp:90-158)
        double sc = 0.0;
        for (auto &p : pairs) {
            const double distance = std::sqrt((0.0 * 0.0 + 0.0 * 0.0) + 0.0 * 0.0);
            const double radii = a.self_collision_radii[p[0] - 3] + a.self_collision_radii[p[1] - 3];
            sc += left_barrier_h(a.self_collision_limit, distance - radii);
        }
        c.self_collision = sc;
        c.ws_above = devb(a.workspace_limit_above);
        c.ws_infront = devb(a.workspace_limit_infront);
        c.ws_reach = devb(a.workspace_limit_reach);
        c.yaw_c = a.workspace_cost_yaw.constant_cost;
        c.yaw_l = a.workspace_cost_yaw.linear_cost;
        c.yaw_q = a.workspace_cost_yaw.quadratic_cost;
        c.manip_c = a.manipulability_cost.constant_cost;
        c.manip_l = a.manipulability_cost.linear_cost;
        c.manip_q = a.manipulability_cost.quadratic_cost;
        c.traj_vel_c = a.trajectory_velocity_cost.constant_cost;
        c.traj_vel_l = a.trajectory_velocity_cost.linear_cost;
        c.traj_vel_q = a.trajectory_velocity_cost.quadratic_cost;
    }
}

mppi_status check_topology(const mppi_frankaridgeback_desc &d, std::string &why)
{
    if (d.nbodies != FR_NB) { why = "frankaridgeback model must have 12 bodies"; return MPPI_ERR_UNSUPPORTED; }
    for (int i = 0; i < FR_NB; i++) {
        const mppi_body &b = d.bodies[i];
        if (b.parent != FR_PARENT[i]) { why = "body " + std::to_string(i) + " parent does not match the FrankaRidgeback topology"; return MPPI_ERR_UNSUPPORTED; }
        const double *a = b.axis;
        bool ok = false;
        switch (FR_KIND[i]) {
        case KIND_PX: ok = b.type == MPPI_JOINT_PRISMATIC && a[0] == 1 && a[1] == 0 && a[2] == 0; break;
        case KIND_PY: ok = b.type == MPPI_JOINT_PRISMATIC && a[0] == 0 && a[1] == 1 && a[2] == 0; break;
        case KIND_PNY: ok = b.type == MPPI_JOINT_PRISMATIC && a[0] == 0 && a[1] == -1 && a[2] == 0; break;
        case KIND_RZ: ok = b.type == MPPI_JOINT_REVOLUTE && a[0] == 0 && a[1] == 0 && a[2] == 1; break;
        }
        if (!ok) { why = "body " + std::to_string(i) + " joint type/axis does not match the FrankaRidgeback topology"; return MPPI_ERR_UNSUPPORTED; }
    }
    // The planar base's x / y joints sit unrotated on the world (robot.urdf x_base_joint /
    // y_base_joint, rpy 0 0 0): the solve takes their motion subspaces as the unit axes
    // (column_dots, and the zero M_01 of gj_pivot_0).
    for (int i = 0; i < 2; i++)
        for (int k = 0; k < 9; k++)
            if (d.bodies[i].rotation[k] != ((k % 4 == 0) ? 1.0 : 0.0)) {
                why = "body " + std::to_string(i) + " (planar base joint) placement must be unrotated";
                return MPPI_ERR_UNSUPPORTED;
            }
    // Bodies 2 and 3 (pivot_joint, panda_joint1) turn about z: with z-rotation placements the world
    // poses of bodies 0..3 are a rotation about z and a translation, which the FK scan's last level
    // composes in planar form (fr_coop.hip scan_level_planar8).
    for (int i = 2; i < 4; i++) {
        const double *r = d.bodies[i].rotation;
        if (!(r[2] == 0 && r[5] == 0 && r[6] == 0 && r[7] == 0 && r[8] == 1 && r[0] == r[4] && r[1] == -r[3])) {
            why = "body " + std::to_string(i) + " placement must be a rotation about z";
            return MPPI_ERR_UNSUPPORTED;
        }
    }
    if (d.end_effector.parent != FR_EE_PARENT || d.arm_mount.parent != FR_AM_PARENT) {
        why = "end-effector / arm-mount frame parents do not match the FrankaRidgeback topology";
        return MPPI_ERR_UNSUPPORTED;
    }
    return MPPI_OK;
}

template <class T>
void dfree(mppi_handle *h, T *&p)
{
    if (!p) return;
    (void)hipFree(p);
    h->allocations.erase(std::find(h->allocations.begin(), h->allocations.end(), (void *)p));
    p = nullptr;
}

// The next update's draws made behind the publish (phase 3) so that its sampling launch leaves
// the critical path: device Philox, diagonal transform, an update whose rollout launch runs rounds
// of four-wave workgroups (it copies the kept columns in, FrRolloutArgs::drawn_ahead).
// MPPI_DRAW_AHEAD=0 turns it off (A/B).
static bool draw_ahead_possible(const mppi_handle *h)
{
    if (h->env.draw_ahead_off) return false;
    return h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK && h->C == FR_C && h->tdiag &&
           h->noise_source == MPPI_NOISE_DEVICE_PHILOX && fr_coop_update_fusable(h->count, h->env);
}

// MPPI_TAIL_DRAWS=0: the next update's draws all in rank_draw_kernel behind the publish (A/B)
static bool tail_draws_disabled(const mppi_handle *h)
{
    return h->env.tail_draws_off;
}

mppi_status alloc_shard_buffers(mppi_handle *h)
{
    h->ahead_valid = false;   // the draws ahead live in the buffers freed here
    if (h->d_costs_local) HIP_TRY(hipMemset(h->d_costs_local, 0, (size_t)(h->R + 1) * sizeof(double)));   // a new range
    dfree(h, h->d_noise);
    dfree(h, h->d_noise_prev);
    h->Rpad = std::max<int64_t>(64, (h->count + 63) / 64 * 64);
    HIP_TRY(dalloc(h, &h->d_noise, (size_t)(h->H * h->C * h->Rpad)));
    HIP_TRY(dalloc(h, &h->d_noise_prev, (size_t)(h->H * h->C * h->Rpad)));
    if (h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        dfree(h, h->d_rec);
        HIP_TRY(dalloc(h, &h->d_rec, (size_t)(h->H * h->Rpad * FR_REC)));
    }
    return MPPI_OK;
}

int64_t keep_count(const mppi_handle *h)
{
    int64_t k = h->compat_uint8 ? (int64_t)(uint8_t)h->K : h->K;
    return std::min(k, h->S);
}

int64_t draws_for(const mppi_handle *h, int64_t shift_by)
{
    const int64_t keep = keep_count(h);
    int64_t d = (h->S - keep) * h->H;
    if (shift_by > 0) d += keep * std::min<int64_t>(shift_by, h->H);
    return d;
}

}  // namespace

// ---- FrankaRidgeback::PinocchioDynamics as a device object (fr_object.hip) --------------------

struct mppi_dynamics {
    int device = 0;
    hipStream_t stream = nullptr;
    DevModel *d_model = nullptr;
    DevPinocchio *d_obj = nullptr;
    double *d_buf = nullptr;   // forecast rows / cost output / wrench rows
    size_t buf_doubles = 0;
    DevPinocchio *h_obj = nullptr;   // pinned host copy for the queries
    std::string err;
};

namespace {

mppi_status dfail(mppi_dynamics *d, mppi_status st, const std::string &msg)
{
    if (d) d->err = msg;
    g_last_error = msg;
    return st;
}

#define DHIP_TRY(expr)                                                                                         \
    do {                                                                                                       \
        hipError_t e_ = (expr);                                                                                \
        if (e_ != hipSuccess) return dfail(d, MPPI_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

DevModel dev_model(const mppi_frankaridgeback_desc &d)
{
    DevModel m{};
    for (int i = 0; i < FR_NB; i++) {
        const mppi_body &b = d.bodies[i];
        std::memcpy(m.b[i].R, b.rotation, sizeof(m.b[i].R));
        std::memcpy(m.b[i].p, b.translation, sizeof(m.b[i].p));
        m.b[i].mass = b.mass;
        std::memcpy(m.b[i].c, b.lever, sizeof(m.b[i].c));
        std::memcpy(m.b[i].Ic, b.inertia, sizeof(m.b[i].Ic));
    }
    std::memcpy(m.ee_R, d.end_effector.rotation, sizeof(m.ee_R));
    std::memcpy(m.ee_p, d.end_effector.translation, sizeof(m.ee_p));
    std::memcpy(m.am_R, d.arm_mount.rotation, sizeof(m.am_R));
    std::memcpy(m.am_p, d.arm_mount.translation, sizeof(m.am_p));
    const double *R10 = m.b[10].R, *R11 = m.b[11].R, *p10 = m.b[10].p, *p11 = m.b[11].p;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) m.f11_R[3 * r + c] = (R10[r] * R11[c] + R10[3 + r] * R11[3 + c]) + R10[6 + r] * R11[6 + c];
        m.f11_p[r] = (R10[r] * (p11[0] - p10[0]) + R10[3 + r] * (p11[1] - p10[1])) + R10[6 + r] * (p11[2] - p10[2]);
    }
    for (int k = 0; k < 3; k++) m.gravity[k] = d.gravity[k];
    return m;
}

mppi_status obj_buffer(mppi_dynamics *d, size_t doubles)
{
    if (doubles <= d->buf_doubles) return MPPI_OK;
    if (d->d_buf) (void)hipFree(d->d_buf);
    d->d_buf = nullptr;
    d->buf_doubles = 0;
    DHIP_TRY(hipMalloc(&d->d_buf, doubles * sizeof(double)));
    d->buf_doubles = doubles;
    return MPPI_OK;
}

mppi_status obj_run(mppi_dynamics *d, ObjArgs &a)
{
    DHIP_TRY(hipSetDevice(d->device));
    a.obj = d->d_obj;
    a.model = d->d_model;
    DHIP_TRY(launch_fr_object(a, d->stream));
    return MPPI_OK;
}

mppi_status obj_fetch(mppi_dynamics *d)
{
    DHIP_TRY(hipMemcpyAsync(d->h_obj, d->d_obj, sizeof(DevPinocchio), hipMemcpyDeviceToHost, d->stream));
    DHIP_TRY(hipStreamSynchronize(d->stream));
    return MPPI_OK;
}

}  // namespace

extern "C" {

mppi_status mppi_dynamics_create(const mppi_dynamics_desc *desc, const double *initial_state, int device, mppi_dynamics **out)
{
    mppi_dynamics *d = nullptr;
    if (!desc || !initial_state || !out) return dfail(nullptr, MPPI_ERR_INVALID, "null argument");
    *out = nullptr;
    if (desc->kind != MPPI_DYNAMICS_FRANKARIDGEBACK)
        return dfail(nullptr, MPPI_ERR_UNSUPPORTED, "the dynamics object is FrankaRidgeback::PinocchioDynamics only");
    std::string why;
    if (check_topology(desc->frankaridgeback, why) != MPPI_OK) return dfail(nullptr, MPPI_ERR_UNSUPPORTED, why);
    d = new mppi_dynamics();
    d->device = device;
    auto bail = [&](mppi_status st) {
        std::string m = d->err;
        mppi_dynamics_destroy(d);
        return dfail(nullptr, st, m);
    };
#define DCREATE_TRY(expr)                                                                                        \
    do {                                                                                                         \
        hipError_t e_ = (expr);                                                                                  \
        if (e_ != hipSuccess) { d->err = std::string(#expr ": ") + hipGetErrorString(e_); return bail(MPPI_ERR_DEVICE); } \
    } while (0)
    DCREATE_TRY(hipSetDevice(device));
    DCREATE_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    DCREATE_TRY(hipMalloc(&d->d_model, sizeof(DevModel)));
    DCREATE_TRY(hipMalloc(&d->d_obj, sizeof(DevPinocchio)));
    DCREATE_TRY(hipHostMalloc((void **)&d->h_obj, sizeof(DevPinocchio), hipHostMallocDefault));
    const DevModel m = dev_model(desc->frankaridgeback);
    DCREATE_TRY(hipMemcpy(d->d_model, &m, sizeof(m), hipMemcpyHostToDevice));
    DCREATE_TRY(hipMemset(d->d_obj, 0, sizeof(DevPinocchio)));   // the constructor's setZero()s (:106-109)
    DCREATE_TRY(hipDeviceSynchronize());
#undef DCREATE_TRY
    if (mppi_dynamics_set_state(d, initial_state, 0.0) != MPPI_OK) return bail(MPPI_ERR_DEVICE);
    *out = d;
    return MPPI_OK;
}

void mppi_dynamics_destroy(mppi_dynamics *d)
{
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    if (d->d_buf) (void)hipFree(d->d_buf);
    if (d->d_obj) (void)hipFree(d->d_obj);
    if (d->d_model) (void)hipFree(d->d_model);
    if (d->h_obj) (void)hipHostFree(d->h_obj);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

mppi_status mppi_dynamics_set_state(mppi_dynamics *d, const double *state, double time)
{
    if (!d || !state) return MPPI_ERR_INVALID;
    ObjArgs a{};
    a.op = OBJ_SET_STATE;
    std::memcpy(a.x, state, FR_X * sizeof(double));
    a.time = time;
    mppi_status st = obj_run(d, a);
    if (st != MPPI_OK) return st;
    DHIP_TRY(hipStreamSynchronize(d->stream));
    return MPPI_OK;
}

mppi_status mppi_dynamics_step(mppi_dynamics *d, const double *control, double dt, double *state_out)
{
    if (!d || !control) return MPPI_ERR_INVALID;
    ObjArgs a{};
    a.op = OBJ_STEP;
    std::memcpy(a.u, control, FR_C * sizeof(double));
    a.dt = dt;
    mppi_status st = obj_run(d, a);
    if (st != MPPI_OK) return st;
    if (!state_out) {
        DHIP_TRY(hipStreamSynchronize(d->stream));
        return MPPI_OK;
    }
    st = obj_fetch(d);
    if (st != MPPI_OK) return st;
    std::memcpy(state_out, d->h_obj->state, FR_X * sizeof(double));
    return MPPI_OK;
}

mppi_status mppi_dynamics_get_state(mppi_dynamics *d, double *state)
{
    if (!d || !state) return MPPI_ERR_INVALID;
    mppi_status st = obj_fetch(d);
    if (st != MPPI_OK) return st;
    std::memcpy(state, d->h_obj->state, FR_X * sizeof(double));
    return MPPI_OK;
}

mppi_status mppi_dynamics_end_effector(mppi_dynamics *d, double *ee)
{
    if (!d || !ee) return MPPI_ERR_INVALID;
    mppi_status st = obj_fetch(d);
    if (st != MPPI_OK) return st;
    std::memcpy(ee, d->h_obj->ee, MPPI_EE_N * sizeof(double));
    return MPPI_OK;
}

mppi_status mppi_dynamics_query(mppi_dynamics *d, double *out)
{
    if (!d || !out) return MPPI_ERR_INVALID;
    mppi_status st = obj_fetch(d);
    if (st != MPPI_OK) return st;
    const DevPinocchio &P = *d->h_obj;
    std::memcpy(out, P.q, FR_NB * sizeof(double));
    std::memcpy(out + 12, P.v, FR_NB * sizeof(double));
    std::memcpy(out + 24, P.a, FR_NB * sizeof(double));
    std::memcpy(out + 36, P.tau, FR_NB * sizeof(double));
    out[48] = P.energy;
    out[49] = P.power;
    out[50] = P.time;
    std::memcpy(out + 51, P.am, 3 * sizeof(double));
    return MPPI_OK;
}

mppi_status mppi_dynamics_forecast(mppi_dynamics *d, const double *state, double time, double time_step, int64_t steps,
                                   const double *wrench, double *out)
{
    if (!d || !state || !out || steps < 0) return MPPI_ERR_INVALID;
    if (steps == 0) return MPPI_OK;
    const size_t rows = (size_t)steps * MPPI_DF_N, wrows = wrench ? (size_t)steps * 6 : 0;
    mppi_status st = obj_buffer(d, rows + wrows);
    if (st != MPPI_OK) return st;
    ObjArgs a{};
    a.op = OBJ_FORECAST;
    std::memcpy(a.x, state, FR_X * sizeof(double));
    a.time = time;
    a.dt = time_step;
    a.steps = steps;
    a.out = d->d_buf;
    if (wrench) {
        DHIP_TRY(hipMemcpyAsync(d->d_buf + rows, wrench, wrows * sizeof(double), hipMemcpyHostToDevice, d->stream));
        a.wrench = d->d_buf + rows;
    }
    st = obj_run(d, a);
    if (st != MPPI_OK) return st;
    DHIP_TRY(hipMemcpyAsync(out, d->d_buf, rows * sizeof(double), hipMemcpyDeviceToHost, d->stream));
    DHIP_TRY(hipStreamSynchronize(d->stream));
    return MPPI_OK;
}

mppi_status mppi_cost_evaluate(const mppi_cost_desc *cost, mppi_dynamics *d, const double *state, const double *control,
                               const double *wrench6, double *out8)
{
    if (!cost || !d || !state || !out8) return MPPI_ERR_INVALID;
    (void)control;   // neither objective reads the control (assisted_manipulation.cpp:37-72, track_point.cpp:10-34)
    if (cost->kind != MPPI_COST_ASSISTED_MANIPULATION && cost->kind != MPPI_COST_TRACK_POINT)
        return dfail(d, MPPI_ERR_UNSUPPORTED, "get_cost on the device: AssistedManipulation or TrackPoint");
    mppi_status st = obj_buffer(d, 8);
    if (st != MPPI_OK) return st;
    ObjArgs a{};
    a.op = OBJ_COST;
    std::memcpy(a.x, state, FR_X * sizeof(double));
    build_dev_cost(*cost, a.cost);
    const double zero[3] = {0, 0, 0};
    a.sc = step_const(cost->assisted_manipulation, wrench6 ? wrench6 : zero, wrench6 != nullptr, 1.0);
    a.out = d->d_buf;
    st = obj_run(d, a);
    if (st != MPPI_OK) return st;
    DHIP_TRY(hipMemcpyAsync(out8, d->d_buf, 8 * sizeof(double), hipMemcpyDeviceToHost, d->stream));
    DHIP_TRY(hipStreamSynchronize(d->stream));
    return MPPI_OK;
}

}  // extern "C"

extern "C" {

int mppi_abi_version(void) { return MPPI_AMD_ABI_VERSION; }

const char *mppi_build_info(void)
{
    return "mppi_amd: gfx950 HIP kernels (fp64 rollout, one lane per rollout, LDS ABA stack), RCCL sharding";
}

void mppi_default_frankaridgeback(mppi_frankaridgeback_desc *out) { mppi_frankaridgeback_model(out); }
void mppi_default_assisted_manipulation(mppi_assisted_manipulation_desc *out) { mppi_assisted_manipulation_default(out); }
void mppi_default_track_point(mppi_track_point_desc *out) { mppi_track_point_default(out); }

const char *mppi_last_error(const mppi_handle *h) { return h ? h->err.c_str() : g_last_error.c_str(); }

mppi_status mppi_shard_range(int64_t rollout_count, int world, int rank, int64_t *begin, int64_t *end)
{
    if (world < 1 || rank < 0 || rank >= world || rollout_count < 2 * (int64_t)world || !begin || !end)
        return MPPI_ERR_INVALID;
    // contiguous blocks, the first (R mod world) ranks one larger (the reference's ThreadPool
    // partition, mppi.cpp:277-302); rollouts 0 and 1 always land on rank 0.
    const int64_t each = rollout_count / world, extra = rollout_count % world;
    const int64_t b = (int64_t)rank * each + std::min<int64_t>(rank, extra);
    *begin = b;
    *end = b + each + (rank < extra ? 1 : 0);
    return MPPI_OK;
}

mppi_status mppi_create(const mppi_config *cfg, const mppi_dynamics_desc *dyn, const mppi_cost_desc *cost, int device,
                        mppi_handle **out)
{
    mppi_handle *h = nullptr;
    if (!cfg || !dyn || !cost || !out) return fail(nullptr, MPPI_ERR_INVALID, "null argument");
    *out = nullptr;
    const EnvSwitches env = env_switches_read();   // the A/B switches, as the environment holds them now
    const int64_t Cd = dyn->kind == MPPI_DYNAMICS_POINT_MASS ? 3 : (dyn->kind == MPPI_DYNAMICS_FRANKARIDGEBACK ? FR_C : -1);
    const int64_t Xd = dyn->kind == MPPI_DYNAMICS_POINT_MASS ? 6 : FR_X;
    const bool fr_cost = cost->kind == MPPI_COST_ASSISTED_MANIPULATION || cost->kind == MPPI_COST_TRACK_POINT;
    const int64_t Cc = cost->kind == MPPI_COST_QUADRATIC ? 3 : (fr_cost ? FR_C : -2);
    const int64_t Xc = cost->kind == MPPI_COST_QUADRATIC ? 6 : FR_X;
    // Trajectory::create validation, in the reference's order (mppi.cpp:17-69)
    if (Cd < 0) return fail(nullptr, MPPI_ERR_INVALID, "unknown dynamics kind");
    if (Cc < 0) return fail(nullptr, MPPI_ERR_INVALID, "unknown cost kind");
    if (Cd != Cc) return fail(nullptr, MPPI_ERR_INVALID, "controller dynamics control dof " + std::to_string(Cd) + " != cost control dof " + std::to_string(Cc));
    if (Xd != Xc) return fail(nullptr, MPPI_ERR_INVALID, "controller dynamics state dof " + std::to_string(Xd) + " != cost state dof " + std::to_string(Xc));
    if (cfg->control_dof != Cd || !cfg->control_min || !cfg->control_max)
        return fail(nullptr, MPPI_ERR_INVALID, "controller maximum and minimum must have length " + std::to_string(Cd));
    if (!cfg->covariance) return fail(nullptr, MPPI_ERR_INVALID, "controller covariance matrix not square");
    if (cfg->state_dof != Xd || !cfg->initial_state) return fail(nullptr, MPPI_ERR_INVALID, "initial state must have length " + std::to_string(Xd));
    if (cfg->rollouts < 1) return fail(nullptr, MPPI_ERR_INVALID, "trajectory rollouts must be greater than zero");
    if (cfg->keep_best_rollouts < 0) return fail(nullptr, MPPI_ERR_INVALID, "trajectory cached rollouts cannot be less than zero");
    if (cfg->threads <= 0) return fail(nullptr, MPPI_ERR_INVALID, "trajectory threads must be positive nonzero");
    if (cfg->keep_best_rollouts > cfg->rollouts)
        return fail(nullptr, MPPI_ERR_INVALID, "keep_best_rollouts > rollouts (std::span::first out of range in the reference)");
    if (!(cfg->time_step > 0) || !(cfg->horison > 0)) return fail(nullptr, MPPI_ERR_INVALID, "time_step and horison must be positive");
    if (cfg->has_smoothing && (cfg->smoothing_window < 1)) return fail(nullptr, MPPI_ERR_INVALID, "smoothing window must be >= 1");
    std::string why;
    if (dyn->kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        mppi_status st = check_topology(dyn->frankaridgeback, why);
        if (st != MPPI_OK) return fail(nullptr, st, why);
    }

    h = new mppi_handle();
    h->env = env;
    {
        const char *e = getenv("MPPI_HOST_TRACE");
        h->host_trace = e && e[0] == '1';
        // the hipGraph path (mppi_set_graph) is opt-in: at 4096 x 64 it measured 0.2895 ms/update
        // against 0.2820 with eager launches (same box, profiles/r03_graph_ab/)
        const char *g = getenv("MPPI_GRAPH");
        h->graph_mode = g && g[0] == '1' ? 1 : 0;
    }
    h->device = device;
    h->dyn_kind = dyn->kind;
    h->cost_kind = cost->kind;
    h->S = cfg->rollouts;
    h->K = cfg->keep_best_rollouts;
    h->R = h->S + 2;
    h->dt = cfg->time_step;
    h->H = (int64_t)std::ceil(cfg->horison / cfg->time_step);
    h->C = Cd;
    h->X = Xd;
    h->gradient_step = cfg->gradient_step;
    h->cost_scale = cfg->cost_scale;
    h->gamma = cfg->cost_discount_factor;
    h->control_bound = cfg->control_bound;
    h->cmin.assign(cfg->control_min, cfg->control_min + Cd);
    h->cmax.assign(cfg->control_max, cfg->control_max + Cd);
    h->has_default = cfg->has_control_default != 0 && cfg->control_default;
    if (h->has_default) h->cdefault.assign(cfg->control_default, cfg->control_default + Cd);
    h->init_state.assign(cfg->initial_state, cfg->initial_state + Xd);
    h->sg_window = cfg->has_smoothing ? (int)cfg->smoothing_window : 0;
    h->sg_order = cfg->has_smoothing ? (int)cfg->smoothing_order : 0;
    h->am = cost->assisted_manipulation;
    h->quad = cost->quadratic;
    h->pm_mass = dyn->point_mass.mass;
    h->begin = 0;
    h->count = h->R;
    h->U_host.assign((size_t)(h->H * h->C), 0.0);
    if (const char *tp = std::getenv("MPPI_WAVE_TRACE")) h->trace_path = tp;
    noise_transform((int)Cd, cfg->covariance, h->T, h->tdiag);
    if (h->H < 1 || h->H > (1 << 20)) { delete h; return fail(nullptr, MPPI_ERR_INVALID, "horizon steps out of range"); }

    auto cleanup_fail = [&](mppi_status st) {
        std::string m = h->err;
        mppi_destroy(h);
        return fail(nullptr, st, m);
    };
#define CREATE_TRY(expr)                                                                                     \
    do {                                                                                                     \
        hipError_t e_ = (expr);                                                                              \
        if (e_ != hipSuccess) { h->err = std::string(#expr ": ") + hipGetErrorString(e_); return cleanup_fail(MPPI_ERR_DEVICE); } \
    } while (0)

    CREATE_TRY(hipSetDevice(device));
    {
        int ncu = 0, lds = 0;
        CREATE_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        CREATE_TRY(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
        h->env.cus = (unsigned)ncu;   // this handle's device (no process-global: ADVICE r05)
        h->env.lds_max = lds;
    }
    // the update stream at the greatest priority (its queue's dispatches go first): measured
    // 0.7-1.4 us per update faster over seven interleaved pairs at 4096x64
    if (!h->env.stream_prio_off) {
        int lo = 0, hi = 0;
        CREATE_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CREATE_TRY(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi));
    } else {
        CREATE_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    }
    CREATE_TRY(hipStreamCreateWithFlags(&h->stream_opt, hipStreamNonBlocking));
    // timing-only events without the system-scope fence: with it each record held the next kernel
    // on the stream back by ~6 us (cache write-back and invalidate); the host reads nothing they guard
    for (auto &e : h->ev) CREATE_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_pub, hipEventDisableTiming));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_opt_done, hipEventDisableTiming));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_opt_end, hipEventDisableSystemFence));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_dyn, hipEventDisableSystemFence));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_wg, hipEventDisableSystemFence));
    CREATE_TRY(hipEventCreateWithFlags(&h->ev_ar, hipEventDisableSystemFence));
    const size_t HC = (size_t)(h->H * h->C);
    CREATE_TRY(dalloc(h, &h->d_x0, (size_t)Xd));
    CREATE_TRY(dalloc(h, &h->d_x0_opt, (size_t)Xd));
    CREATE_TRY(dalloc(h, &h->d_U, HC));
    CREATE_TRY(dalloc(h, &h->d_Us, HC));
    CREATE_TRY(dalloc(h, &h->d_costs, (size_t)h->R + 1));   // + slot R: the all-reduced wait timeouts
    CREATE_TRY(dalloc(h, &h->d_gpart, HC));
    CREATE_TRY(dalloc(h, &h->d_grad, HC));
    CREATE_TRY(dalloc(h, &h->d_gsplit, HC * GRAD_SPLIT));
    CREATE_TRY(dalloc(h, &h->d_wexp, (size_t)h->R));
    CREATE_TRY(dalloc(h, &h->d_cstats, 1));
    // the first update's statistics start empty (later ones are reset by the finish kernel)
    CREATE_TRY(hipMemset(h->d_cstats->kmin, 0xFF, sizeof(h->d_cstats->kmin)));
    CREATE_TRY(dalloc(h, &h->d_wpart, 4 * 64));
    CREATE_TRY(dalloc(h, &h->d_T, (size_t)(Cd * Cd)));
    CREATE_TRY(dalloc(h, &h->d_opt, 1));
    CREATE_TRY(dalloc(h, &h->d_rec_opt, (size_t)(h->H * FR_REC)));
    if (dyn->kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {   // the relay's hand-off slots; tokens start at 0 (never a launch's)
        CREATE_TRY(dalloc(h, &h->d_rx, (size_t)RELAY_GROUPS_MAX));
        CREATE_TRY(hipMemset(h->d_rx, 0, sizeof(RelayXfer) * RELAY_GROUPS_MAX));
    }
    CREATE_TRY(dalloc(h, &h->d_cmin, (size_t)Cd));
    CREATE_TRY(dalloc(h, &h->d_cmax, (size_t)Cd));
    CREATE_TRY(dalloc(h, &h->d_rank, (size_t)h->R));
    CREATE_TRY(dalloc(h, &h->d_rank_keys, (size_t)rank_scratch(h->S)));
    CREATE_TRY(dalloc(h, &h->d_status, 1));
    CREATE_TRY(dalloc(h, &h->d_steps_buf[0], (size_t)h->H));
    CREATE_TRY(dalloc(h, &h->d_steps_buf[1], (size_t)h->H));
    h->d_steps = h->d_steps_buf[0];
    CREATE_TRY(dalloc(h, &h->d_gamma, (size_t)h->H));
    CREATE_TRY(dalloc(h, &h->d_fc_out, 6));
    CREATE_TRY(dalloc(h, &h->d_terms, 7));
    {
        std::vector<double> g((size_t)h->H);
        for (int64_t k = 0; k < h->H; k++) g[(size_t)k] = std::pow(h->gamma, (double)k);
        CREATE_TRY(hipMemcpy(h->d_gamma, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    CREATE_TRY(hipHostMalloc((void **)&h->h_out, (HC + 8) * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    CREATE_TRY(hipHostGetDevicePointer((void **)&h->h_out_dev, h->h_out, 0));
    std::memset(h->h_out, 0, (HC + 8) * sizeof(double));   // the publish flag starts below every sequence
    CREATE_TRY(hipHostMalloc((void **)&h->h_opt, 8 * sizeof(double), hipHostMallocDefault));
    h->h_opt[0] = 0.0;
    CREATE_TRY(hipMemcpy(h->d_T, h->T.data(), h->T.size() * sizeof(double), hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_cmin, h->cmin.data(), (size_t)Cd * sizeof(double), hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_cmax, h->cmax.data(), (size_t)Cd * sizeof(double), hipMemcpyHostToDevice));
    CREATE_TRY(hipMemcpy(h->d_x0, h->init_state.data(), (size_t)Xd * sizeof(double), hipMemcpyHostToDevice));

    if (dyn->kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        DevModel m{};
        const mppi_frankaridgeback_desc &d = dyn->frankaridgeback;
        for (int i = 0; i < FR_NB; i++) {
            const mppi_body &b = d.bodies[i];
            std::memcpy(m.b[i].R, b.rotation, sizeof(m.b[i].R));
            std::memcpy(m.b[i].p, b.translation, sizeof(m.b[i].p));
            m.b[i].mass = b.mass;
            std::memcpy(m.b[i].c, b.lever, sizeof(m.b[i].c));
            std::memcpy(m.b[i].Ic, b.inertia, sizeof(m.b[i].Ic));
        }
        std::memcpy(m.ee_R, d.end_effector.rotation, sizeof(m.ee_R));
        std::memcpy(m.ee_p, d.end_effector.translation, sizeof(m.ee_p));
        std::memcpy(m.am_R, d.arm_mount.rotation, sizeof(m.am_R));
        std::memcpy(m.am_p, d.arm_mount.translation, sizeof(m.am_p));
        {
            const double *R10 = m.b[10].R, *R11 = m.b[11].R, *p10 = m.b[10].p, *p11 = m.b[11].p;
            for (int r = 0; r < 3; r++) {
                for (int c = 0; c < 3; c++)
                    m.f11_R[3 * r + c] = (R10[r] * R11[c] + R10[3 + r] * R11[3 + c]) + R10[6 + r] * R11[6 + c];
                m.f11_p[r] = (R10[r] * (p11[0] - p10[0]) + R10[3 + r] * (p11[1] - p10[1])) + R10[6 + r] * (p11[2] - p10[2]);
            }
        }
        for (int k = 0; k < 3; k++) m.gravity[k] = d.gravity[k];
        CREATE_TRY(dalloc(h, &h->d_model, 1));
        CREATE_TRY(hipMemcpy(h->d_model, &m, sizeof(m), hipMemcpyHostToDevice));
        DevCost c{};
        build_dev_cost(*cost, c);
        CREATE_TRY(dalloc(h, &h->d_cost, 1));
        CREATE_TRY(hipMemcpy(h->d_cost, &c, sizeof(c), hipMemcpyHostToDevice));
        CREATE_TRY(dalloc(h, &h->d_table, FR_BODY_TABLE));
        CREATE_TRY(launch_fr_body_table(h->d_model, h->d_cost, h->d_table, nullptr));
        CREATE_TRY(hipDeviceSynchronize());
    } else {
        DevPointMass p{};
        p.inv_mass = 1.0 / dyn->point_mass.mass;
        for (int i = 0; i < 3; i++) {
            p.target[i] = cost->quadratic.target[i];
            p.q[i] = cost->quadratic.q[i];
            p.r[i] = cost->quadratic.r[i];
        }
        CREATE_TRY(dalloc(h, &h->d_pm, 1));
        CREATE_TRY(hipMemcpy(h->d_pm, &p, sizeof(p), hipMemcpyHostToDevice));
        h->pm_host = p;
        const int rows = pm_fused_rows(h->R, (int)h->H, h->env.cus, h->env.lds_max);
        if (h->C == 3 && h->X == 6 && rows) {   // the one-launch update's scratch
            h->pm_nblocks = (unsigned)((h->R + rows - 1) / rows);
            CREATE_TRY(dalloc(h, &h->d_pm_sync, 2));
            CREATE_TRY(dalloc(h, &h->d_pm_part, (size_t)h->pm_nblocks * (HC + 1)));
            const char *ps = std::getenv("MPPI_PM_STAMPS");
            if (ps && ps[0] == '1') {
                CREATE_TRY(dalloc(h, &h->d_pm_stamps, (size_t)h->pm_nblocks * PM_STAMPS));
                h->pm_stamp_sum.assign(PM_STAMPS, 0.0);
            }
        }
    }
    if (h->sg_window > 0) {
        const int w = h->sg_window;
        const int64_t W = h->H + 2 * w + 1;
        std::vector<double> sw = sg_weights(w, h->sg_order);
        CREATE_TRY(dalloc(h, &h->d_sg_w, sw.size()));
        CREATE_TRY(hipMemcpy(h->d_sg_w, sw.data(), sw.size() * sizeof(double), hipMemcpyHostToDevice));
        CREATE_TRY(dalloc(h, &h->d_sg_uu, (size_t)(h->C * W)));
        CREATE_TRY(dalloc(h, &h->d_sg_tt, (size_t)(h->C * W)));
        std::vector<double> tt((size_t)(h->C * W), -1.0);   // MovingExtendedWindow: tt = -1, uu = 0
        CREATE_TRY(hipMemcpy(h->d_sg_tt, tt.data(), tt.size() * sizeof(double), hipMemcpyHostToDevice));
        CREATE_TRY(dalloc(h, &h->d_sg_start, (size_t)h->C));
        std::vector<int64_t> st((size_t)h->C, (int64_t)w);
        CREATE_TRY(hipMemcpy(h->d_sg_start, st.data(), st.size() * sizeof(int64_t), hipMemcpyHostToDevice));
        CREATE_TRY(dalloc(h, &h->d_sg_last, (size_t)h->C));
        std::vector<double> lt((size_t)h->C, -1.0);
        CREATE_TRY(hipMemcpy(h->d_sg_last, lt.data(), lt.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    {
        mppi_status st = alloc_shard_buffers(h);
        if (st != MPPI_OK) return cleanup_fail(st);
        st = upload_steps(h);
        if (st != MPPI_OK) return cleanup_fail(st);
    }
    // the first update's order: every previous cost is 0 (mppi.cpp:222-231: identity).  The
    // zero-fills above run on the null stream, which the non-blocking streams do not wait for.
    CREATE_TRY(hipDeviceSynchronize());
    CREATE_TRY(launch_rank(h->d_costs, h->S, h->d_rank, h->d_rank_keys, h->stream));
    if (!h->trace_path.empty()) CREATE_TRY(dalloc(h, &h->d_trace, (size_t)(4 * ((h->R + 1) / 4 + 40))));   // + the relay waves' and block 0's chunks' slots (COOP_TRACE)
#undef CREATE_TRY
    *out = h;
    return MPPI_OK;
}

void mppi_destroy(mppi_handle *h)
{
    if (!h) return;
    if (h->pm_stamp_n > 0) {
        std::fprintf(stderr, "pm_update_kernel phases (us after the first block's entry, last block, mean of %lld):",
                     (long long)h->pm_stamp_n);
        static const char *names[PM_STAMPS] = {"entry", "sampled", "rolled", "barrier", "partials", "ticket",
                                               "staged", "stored", "published", "ranked", "end", "costs"};
        for (int i = 0; i < PM_STAMPS; i++) std::fprintf(stderr, " %s %.2f", names[i], h->pm_stamp_sum[(size_t)i] / (double)h->pm_stamp_n);
        std::fprintf(stderr, "\n");
    }
    if (h->host_trace && h->ht_n[2] > 0)
        std::fprintf(stderr, "mppi host turnaround (us): flag->return %.2f  return->phase1 %.2f  phase1->launched %.2f  (n=%lld)\n",
                     h->ht_sum[0] / (double)std::max<int64_t>(1, h->ht_n[0]), h->ht_sum[1] / (double)std::max<int64_t>(1, h->ht_n[1]),
                     h->ht_sum[2] / (double)h->ht_n[2], (long long)h->ht_n[2]);
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->stream_opt) (void)hipStreamSynchronize(h->stream_opt);
    if (h->comm) ncclCommDestroy(h->comm);
    if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    for (void *p : h->allocations) (void)hipFree(p);
    if (h->h_out) (void)hipHostFree(h->h_out);
    if (h->h_opt) (void)hipHostFree(h->h_opt);
    if (h->ev_pub) (void)hipEventDestroy(h->ev_pub);
    if (h->ev_opt_done) (void)hipEventDestroy(h->ev_opt_done);
    if (h->ev_opt_end) (void)hipEventDestroy(h->ev_opt_end);
    if (h->ev_dyn) (void)hipEventDestroy(h->ev_dyn);
    if (h->ev_wg) (void)hipEventDestroy(h->ev_wg);
    if (h->ev_ar) (void)hipEventDestroy(h->ev_ar);
    if (h->stream_opt) (void)hipStreamDestroy(h->stream_opt);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : h->ev_ring)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

// The sharded update path (cost vector and partial gradient all-reduced, the weights from the
// all-reduced costs): world > 1, or a one-rank communicator (mppi_comm_init with world 1), which
// runs the same path through RCCL on one GPU
static inline bool sharded(const mppi_handle *h) { return h->world > 1 || h->comm != nullptr; }

mppi_status mppi_set_shard(mppi_handle *h, int world, int rank)
{
    if (!h) return MPPI_ERR_INVALID;
    if (h->updated_once) return fail(h, MPPI_ERR_INVALID, "shard must be set before the first update");
    int64_t b, e;
    if (mppi_shard_range(h->R, world, rank, &b, &e) != MPPI_OK) return fail(h, MPPI_ERR_INVALID, "invalid shard");
    HIP_TRY(hipSetDevice(h->device));
    h->world = world;
    h->rank = rank;
    h->begin = b;
    h->count = e - b;
    return alloc_shard_buffers(h);
}

mppi_status mppi_comm_unique_id(char out[128])
{
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPPI_ERR_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, 128);
    return MPPI_OK;
}

mppi_status mppi_comm_init(mppi_handle *h, int world, int rank, const char unique_id[128])
{
    if (!h) return MPPI_ERR_INVALID;
    mppi_status st = mppi_set_shard(h, world, rank);
    if (st != MPPI_OK) return st;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, 128);
    HIP_TRY(hipSetDevice(h->device));
    NCCL_TRY(ncclCommInitRank(&h->comm, world, id, rank));
    if (!h->d_costs_local) HIP_TRY(dalloc(h, &h->d_costs_local, (size_t)h->R + 1));   // + the wait-timeout slot
    return MPPI_OK;
}

mppi_status mppi_comm_info(mppi_handle *h, int *nranks, int *rank, int *device, char *pci_bus_id, int len)
{
    if (!h || !nranks || !rank) return MPPI_ERR_INVALID;
    if (h->comm) {   // what the communicator itself says, not what the caller asked for
        NCCL_TRY(ncclCommCount(h->comm, nranks));
        NCCL_TRY(ncclCommUserRank(h->comm, rank));
    } else {
        *nranks = 0;
        *rank = -1;
    }
    if (device) *device = h->device;
    if (pci_bus_id && len > 0) HIP_TRY(hipDeviceGetPCIBusId(pci_bus_id, len, h->device));
    return MPPI_OK;
}

mppi_status mppi_set_noise_source(mppi_handle *h, int source, uint64_t seed)
{
    if (!h || (source != MPPI_NOISE_DEVICE_PHILOX && source != MPPI_NOISE_HOST_INJECTED)) return MPPI_ERR_INVALID;
    h->noise_source = source;
    h->seed = seed;
    return MPPI_OK;
}

mppi_status mppi_inject_noise(mppi_handle *h, const double *eps, int64_t columns)
{
    if (!h || (!eps && columns) || columns < 0) return MPPI_ERR_INVALID;
    h->inj_pending.insert(h->inj_pending.end(), eps, eps + columns * h->C);
    return MPPI_OK;
}

mppi_status mppi_noise_draws(mppi_handle *h, double time, int64_t *columns)
{
    if (!h || !columns) return MPPI_ERR_INVALID;
    *columns = draws_for(h, (int64_t)((time - h->last_shift_time) / h->dt));
    return MPPI_OK;
}

mppi_status mppi_set_index_semantics(mppi_handle *h, int semantics)
{
    if (!h) return MPPI_ERR_INVALID;
    if (semantics == MPPI_INDEX_COMPAT_UINT8) {
        if (h->R > 255) return fail(h, MPPI_ERR_UNSUPPORTED, "compat uint8 index semantics require rollouts + 2 <= 255 (the reference hangs beyond)");
        h->compat_uint8 = 1;
    } else if (semantics == MPPI_INDEX_WIDE) {
        h->compat_uint8 = 0;
    } else {
        return MPPI_ERR_INVALID;
    }
    return MPPI_OK;
}

mppi_status mppi_set_forecast(mppi_handle *h, const double *wrench_Hx6)
{
    if (!h) return MPPI_ERR_INVALID;
    if (wrench_Hx6) h->forecast.assign(wrench_Hx6, wrench_Hx6 + 6 * h->H);
    else h->forecast.clear();
    h->fc.type = FC_NONE;   // a table replaces an attached forecast
    HIP_TRY(hipSetDevice(h->device));
    if (h->opt_state == mppi_handle::OPT_PENDING) {   // the pending filter() reads the old constants
        mppi_status st = launch_filter_standalone(h);
        if (st != MPPI_OK) return st;
    }
    HIP_TRY(hipStreamSynchronize(h->stream_opt));   // the pending optimal rollout reads d_steps
    return upload_steps(h);
}

namespace {

ForecastArgs forecast_args(const mppi_handle *h)
{
    ForecastArgs f{};
    f.type = h->fc.type;
    f.steps = h->fc.steps;
    for (int k = 0; k < 6; k++) f.value[k] = h->fc.value[k];
    f.valid_until = h->fc.valid_until;
    f.last_update = h->fc.last_update;
    f.horison = h->fc.horison;
    f.time_step = h->fc.time_step;
    f.pred = h->fc.d_pred;
    return f;
}

StepParams step_params(const mppi_handle *h)
{
    const mppi_assisted_manipulation_desc &a = h->am;
    StepParams p{};
    p.assisted_manipulation = h->cost_kind == MPPI_COST_ASSISTED_MANIPULATION;
    p.has_forecast = a.has_forecast;
    p.target_scale = a.trajectory_target_scale;
    p.target_maximum = a.trajectory_target_maximum;
    p.position_threshold = a.trajectory_position_threshold;
    p.pos_c = a.trajectory_position_cost.constant_cost;
    p.pos_l = a.trajectory_position_cost.linear_cost;
    p.pos_q = a.trajectory_position_cost.quadratic_cost;
    p.vel_dropoff = a.trajectory_velocity_dropoff;
    p.vel_minimum = a.trajectory_velocity_minimum;
    p.vel_maximum = a.trajectory_velocity_maximum;
    return p;
}

unsigned fc_factorial(unsigned k) { return k <= 1 ? 1 : k * fc_factorial(k - 1); }

// AverageForecast::clear_old_measurements + update_average (forecast.cpp:67-101)
void average_refresh(mppi_handle::DeviceForecast &f, double time)
{
    size_t it = 0;
    while (it < f.buffer.size() && !(time - f.window < f.buffer[it].first)) it++;
    f.buffer.erase(f.buffer.begin(), f.buffer.begin() + (long)it);
    if (f.buffer.empty()) {
        for (double &v : f.value) v = 0.0;
        return;
    }
    std::array<double, 6> total = f.buffer[0].second;
    for (size_t i = 1; i < f.buffer.size(); i++)
        for (int k = 0; k < 6; k++) total[(size_t)k] += f.buffer[i].second[(size_t)k];
    for (int k = 0; k < 6; k++) f.value[k] = total[(size_t)k] / (double)f.buffer.size();
}

}  // namespace

mppi_status mppi_forecast_attach(mppi_handle *h, const mppi_forecast_config *c)
{
    if (!h) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->opt_state == mppi_handle::OPT_PENDING) {   // the pending filter() reads the current constants
        mppi_status st = launch_filter_standalone(h);
        if (st != MPPI_OK) return st;
        HIP_TRY(hipStreamSynchronize(h->stream_opt));
    }
    mppi_handle::DeviceForecast &f = h->fc;
    if (!c) {   // detach: back to the caller's table
        f.type = FC_NONE;
        return upload_steps(h);
    }
    // Forecast::create (forecast.cpp:6-39) and the kind's create()
    if (c->type != MPPI_FORECAST_LOCF && c->type != MPPI_FORECAST_AVERAGE && c->type != MPPI_FORECAST_KALMAN)
        return fail(h, MPPI_ERR_INVALID, "unknown forecast type " + std::to_string(c->type) + "selected");
    dfree(h, f.d_kf);
    dfree(h, f.d_pred);
    if (c->type == MPPI_FORECAST_LOCF) {
        f = mppi_handle::DeviceForecast{};
        for (int k = 0; k < 6; k++) f.value[k] = c->locf_observation[k];
        f.horison = c->locf_horison;
        f.valid_until = 0.0;
    } else if (c->type == MPPI_FORECAST_AVERAGE) {
        if (c->average_window < 0.0) return fail(h, MPPI_ERR_INVALID, "prediction window time is negative");
        if (c->average_states != 6) return fail(h, MPPI_ERR_UNSUPPORTED, "the end-effector wrench forecast has 6 states");
        f = mppi_handle::DeviceForecast{};
        f.window = c->average_window;
    } else if (c->type == MPPI_FORECAST_KALMAN) {
        if (c->kalman_observed_states != 6)
            return fail(h, MPPI_ERR_UNSUPPORTED, "KalmanForecast::update works on the 6-state wrench (forecast.cpp:303)");
        if (c->kalman_order < 0 || c->kalman_order > MPPI_FORECAST_MAX_ORDER)
            return fail(h, MPPI_ERR_UNSUPPORTED, "kalman order must be in [0, " + std::to_string(MPPI_FORECAST_MAX_ORDER) + "]");
        if (!(c->kalman_time_step > 0) || !(c->kalman_horison >= 0))
            return fail(h, MPPI_ERR_INVALID, "kalman time_step must be positive and horison non-negative");
        f = mppi_handle::DeviceForecast{};
        f.order = c->kalman_order;
        f.n = 6 * (f.order + 1);
        f.time_step = c->kalman_time_step;
        f.horison = c->kalman_horison;
        f.steps = (int)std::ceil(c->kalman_horison / c->kalman_time_step);
        f.last_update = -c->kalman_time_step;
        DevKalman k{};
        const int n = f.n;
        for (int d = 0; d <= f.order; d++)   // create_euler_state_transition_matrix (forecast.cpp:238-285)
            for (int st = 0; st < 6; st++)
                for (int i = 0; i <= f.order - d; i++)
                    k.F[(d * 6 + st) * KMAX + d * 6 + i * 6 + st] = 1.0 / (double)fc_factorial((unsigned)i) * std::pow(f.time_step, (double)i);
        for (int i = 0; i < n; i++) k.P[i * KMAX + i] = 1e-8;   // initial_covariance
        for (int i = 0; i < 6; i++) k.x[i] = c->kalman_initial_state[i];
        for (int i = 0; i < n; i++) {   // m_next_state = F x0
            double acc = 0.0;
            for (int j = 0; j < n; j++) acc += k.F[i * KMAX + j] * k.x[j];
            k.xn[i] = acc;
        }
        HIP_TRY(dalloc(h, &f.d_kf, 1));
        HIP_TRY(dalloc(h, &f.d_pred, (size_t)(f.steps + 1) * 6));   // zeros: uninitialised in the reference
        HIP_TRY(hipMemcpy(f.d_kf, &k, sizeof(k), hipMemcpyHostToDevice));
    }
    f.type = c->type;
    return MPPI_OK;
}

mppi_status mppi_forecast_observe(mppi_handle *h, const double *m, double time)
{
    if (!h || !m || h->fc.type == FC_NONE) return MPPI_ERR_INVALID;
    mppi_handle::DeviceForecast &f = h->fc;
    if (f.type == FC_LOCF) {   // forecast.hpp:96-100
        f.valid_until = time + f.horison;
        for (int k = 0; k < 6; k++) f.value[k] = m[k];
    } else if (f.type == FC_AVERAGE) {   // forecast.cpp:109-122
        if (time < f.last) return MPPI_OK;
        f.last = time;
        f.buffer.emplace_back(time, std::array<double, 6>{m[0], m[1], m[2], m[3], m[4], m[5]});
        average_refresh(f, time);
    } else {   // KalmanForecast::update (forecast.cpp:298-331) on the engine stream
        HIP_TRY(hipSetDevice(h->device));
        KalmanObserve a{};
        a.n = f.n;
        a.order = f.order;
        a.steps = f.steps;
        a.pending = f.pending;
        a.dt = time - f.last_update;
        for (int k = 0; k < 6; k++) a.m[k] = m[k];
        HIP_TRY(launch_kalman_observe(f.d_kf, f.d_pred, a, h->stream));
        f.pending = 0;
        f.last_update = time;
    }
    return MPPI_OK;
}

mppi_status mppi_forecast_observe_time(mppi_handle *h, double time)
{
    if (!h || h->fc.type == FC_NONE) return MPPI_ERR_INVALID;
    mppi_handle::DeviceForecast &f = h->fc;
    if (f.type == FC_AVERAGE) {
        average_refresh(f, time);   // forecast.cpp:102-107
    } else if (f.type == FC_KALMAN) {
        // forecast.cpp:333-340: filter predict(); it changes only the filter state, which the next
        // observation reads, so the predictions are applied at the start of that observation
        if (time > f.last_update) f.pending++;
    }
    return MPPI_OK;
}

mppi_status mppi_forecast_get(mppi_handle *h, double time, double *out)
{
    if (!h || !out || h->fc.type == FC_NONE) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(launch_forecast_eval(forecast_args(h), time, h->d_fc_out, h->stream));
    HIP_TRY(hipMemcpyAsync(out, h->d_fc_out, 6 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MPPI_OK;
}

mppi_status mppi_forecast_table(mppi_handle *h, double t0, double dt, int64_t steps, double *out)
{
    if (!h || !out || steps < 0 || h->fc.type == FC_NONE) return MPPI_ERR_INVALID;
    if (steps == 0) return MPPI_OK;
    HIP_TRY(hipSetDevice(h->device));
    double *buf = nullptr;
    // on the engine stream: behind the Kalman observations that write the prediction table
    HIP_TRY(hipMallocAsync((void **)&buf, (size_t)steps * 6 * sizeof(double), h->stream));
    HIP_TRY(launch_forecast_table(forecast_args(h), t0, dt, steps, buf, h->stream));
    HIP_TRY(hipMemcpyAsync(out, buf, (size_t)steps * 6 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipFreeAsync(buf, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MPPI_OK;
}

mppi_status mppi_step_constants(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    std::vector<StepConst> st((size_t)h->H);
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(st.data(), h->d_steps, st.size() * sizeof(StepConst), hipMemcpyDeviceToHost));
    for (size_t k = 0; k < st.size(); k++) {
        double *o = out + 8 * k;
        o[0] = st[k].target[0]; o[1] = st[k].target[1]; o[2] = st[k].target[2];
        o[3] = st[k].tt; o[4] = st[k].pos_cost; o[5] = st[k].vtarget; o[6] = st[k].gamma_k; o[7] = st[k].active;
    }
    return MPPI_OK;
}

void *mppi_device_costs(mppi_handle *h) { return h ? (void *)h->d_costs : nullptr; }
int64_t mppi_device_costs_count(mppi_handle *h) { return h ? h->R + 1 : 0; }
void *mppi_device_gradient(mppi_handle *h) { return h ? (void *)h->d_gpart : nullptr; }
void *mppi_stream(mppi_handle *h) { return h ? (void *)h->stream : nullptr; }

// ---- update ---------------------------------------------------------------------------------

// The cost kernel's view of a cooperative rollout launch (same rows, records and outputs).
// Unsharded cooperative FrankaRidgeback updates take the costs' min / max / count from the cost
// kernel (CostStats); sharded ones see only their own costs there and reduce after the all-reduce.
static bool cost_stats_used(const mppi_handle *h)
{
    return !sharded(h) && h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK;
}

// Where an update's rollout costs go: d_costs, or the rank's zero-padded local vector that the
// engine's own all-reduce sums into d_costs
static double *rollout_costs_out(const mppi_handle *h)
{
    return h->comm ? h->d_costs_local : h->d_costs;
}

// compact: the records are fr_coop_kernel's (FR_REC_C), not fr_coop_x_kernel's (FR_REC)
static FrCostArgs cost_args(const mppi_handle *h, const FrRolloutArgs &a, bool compact)
{
    FrCostArgs c{};
    c.compact = compact ? 1 : 0;
    c.cost = a.cost;
    c.steps = a.steps;
    c.rec = a.rec;
    c.begin = a.begin;
    c.count = a.count;
    c.cost_out = a.cost_out;
    c.status = a.status;
    c.H = a.H;
    c.optimal = a.optimal;
    c.cost_kind = a.cost_kind;
    c.energy = a.energy;
    c.frec = a.frec;
    c.fsteps = a.fsteps;
    c.fcost = a.fcost;
    c.stats = cost_stats_used(h) ? h->d_cstats : nullptr;
    return c;
}

// filter() of the last update on the side stream, by itself (mppi.cpp:450-479)
static mppi_status launch_filter_standalone(mppi_handle *h)
{
    // cooperative FrankaRidgeback: phase 3 left filter() pending (it rides in the next rollout
    // launch) and recorded no event behind the finish kernel, to keep one off the update path; the
    // row reads the d_U / d_x0_opt that kernel wrote, so order the side stream behind it now
    // (the fused point-mass launch leaves it pending the same way; elsewhere phase 3 recorded the
    // event just before, and recording it again marks the same point of the stream)
    HIP_TRY(hipEventRecord(h->ev_pub, h->stream));
    HIP_TRY(hipStreamWaitEvent(h->stream_opt, h->ev_pub, 0));
    HIP_TRY(hipEventRecord(h->ev[4], h->stream_opt));
    if (h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        FrRolloutArgs a{};
        a.model = h->d_model;
        a.cost = h->d_cost;
        a.table = h->d_table;
        a.steps = h->opt_steps;
        a.x0 = h->d_x0_opt;
        a.Ushift = h->d_U;
        a.cost_out = h->d_opt;
        a.status = h->d_status;
        a.count = 1;
        a.Rpad = 64;
        a.dt = h->dt;
        a.H = (int)h->H;
        a.optimal = 1;
        a.cost_kind = h->cost_kind;
        a.energy = h->cost_kind == MPPI_COST_ASSISTED_MANIPULATION && h->am.enable_energy_limit;
        a.rec = h->d_rec_opt;
        // the row's objective after its loop (fr_coop_kernel's one-wave path)
        a.costs_in_launch = fr_coop_costs_in_launch(h->env) ? 1 : 0;
        HIP_TRY(launch_fr_coop(a, h->stream_opt));
        const bool compact = fr_coop_compact(a);   // (false: the standalone row keeps the 768-B record)
        if (!a.costs_in_launch) HIP_TRY(launch_fr_step_cost(cost_args(h, a, compact), h->stream_opt));
        h->opt_rec_compact = compact;
    } else {
        PmRolloutArgs a{};
        a.pm = h->d_pm;
        a.steps = h->opt_steps;
        a.x0 = h->d_x0_opt;
        a.Ushift = h->d_U;
        a.cost_out = h->d_opt;
        a.status = h->d_status;
        a.count = 1;
        a.Rpad = 64;
        a.dt = h->dt;
        a.H = (int)h->H;
        a.optimal = 1;
        HIP_TRY(launch_pm_rollout(a, h->stream_opt));
    }
    HIP_TRY(hipEventRecord(h->ev_opt_end, h->stream_opt));
    HIP_TRY(hipMemcpyAsync(h->h_opt, h->d_opt, sizeof(double), hipMemcpyDeviceToHost, h->stream_opt));
    HIP_TRY(hipEventRecord(h->ev_opt_done, h->stream_opt));
    h->opt_state = mppi_handle::OPT_LAUNCHED;
    return MPPI_OK;
}

static WGradArgs wgrad_args(const mppi_handle *h);
static FinishArgs finish_args(mppi_handle *h);

mppi_status mppi_update_phase1(mppi_handle *h, const double *state, double time)
{
    if (!h || !state) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    h->t_start = std::chrono::steady_clock::now();
    h->tail_drawn = false;
    if (h->host_trace && h->ht_n[0] > h->ht_n[1]) {
        h->ht_sum[1] += std::chrono::duration<double, std::micro>(h->t_start - h->ht_ret).count();
        h->ht_n[1]++;
    }
    h->rollout_time = time;
    if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev[0], h->stream));
    if (h->fc.type != FC_NONE) {   // this update's forecast samples, t0 + k dt (mppi.cpp:326)
        h->d_steps = h->d_steps_buf[(h->update_count + 1) & 1];   // the previous filter() reads the other
        HIP_TRY(launch_forecast_steps(forecast_args(h), step_params(h), h->d_gamma, (int)h->H, time, h->dt, h->d_steps, h->stream));
    }

    // sample(): shift count by truncation (mppi.cpp:194-201)
    h->shift_by = (int64_t)((time - h->last_shift_time) / h->dt);
    if (h->shift_by > 0) {
        h->last_shift_time = time;
        h->shifted = std::max<int64_t>(0, h->H - h->shift_by);
    }
    SampleParams sp{};
    sp.shift_by = h->shift_by;
    sp.shifted = h->shift_by > 0 ? h->shifted : h->H;
    sp.keep = keep_count(h);
    sp.keep_draws = h->shift_by > 0 ? sp.keep * (h->H - h->shifted) : 0;
    sp.update_index = h->update_count;
    sp.seed = h->seed;
    sp.injected = h->noise_source == MPPI_NOISE_HOST_INJECTED;
    sp.tdiag = h->tdiag ? 1 : 0;
    if (sp.injected) {
        const int64_t draws = draws_for(h, h->shift_by);
        const size_t need = (size_t)(draws * h->C);
        if (h->inj_pending.size() < need) return fail(h, MPPI_ERR_NOISE, "injected noise stream too short: need " + std::to_string(draws) + " columns");
        if (need > h->inj_capacity) {
            dfree(h, h->d_inj);
            HIP_TRY(dalloc(h, &h->d_inj, need));
            h->inj_capacity = need;
        }
        if (need) HIP_TRY(hipMemcpy(h->d_inj, h->inj_pending.data(), need * sizeof(double), hipMemcpyHostToDevice));
        h->inj_pending.erase(h->inj_pending.begin(), h->inj_pending.begin() + (long)need);
    }
    // the stable order of the previous costs was ranked behind the previous publish (phase 3)
    // phase-split callers all-reduce d_costs in place: clear the other ranks' slots first
    // (R + 1: slot R carries the ranks' in-launch wait timeouts, which the caller all-reduces too)
    if (h->world > 1 && !h->comm) HIP_TRY(hipMemsetAsync(h->d_costs, 0, (size_t)(h->R + 1) * sizeof(double), h->stream));
    // this update's draws were made ahead (behind the previous publish) when nothing they depend
    // on changed since; else the cooperative update launch may sample its own rows (opt-in)
    const bool ahead = h->ahead_valid && draw_ahead_possible(h) && h->ahead.update_index == h->update_count &&
                       h->ahead.seed == h->seed && h->ahead.begin == h->begin && h->ahead.count == h->count &&
                       h->ahead.H == h->H && h->ahead.C == h->C;
    h->ahead_valid = false;
    SampleArgs sa{};
    {   // eps of this update into the other buffer; the kept rollouts read the previous one
        std::swap(h->d_noise, h->d_noise_prev);
        sa.rank = h->d_rank;
        sa.Uprev = h->d_U;
        sa.inj = h->d_inj;
        sa.T = h->d_T;
        sa.prev = h->d_noise_prev;
        sa.noise = h->d_noise;
        sa.Us = h->d_Us;
        sa.sp = sp;
        sa.begin = h->begin;
        sa.count = h->count;
        sa.Rpad = h->Rpad;
        sa.H = (int)h->H;
        sa.C = (int)h->C;
        std::memcpy(sa.x0v, state, (size_t)h->X * sizeof(double));   // the state rides in the launch
        sa.x0_out = h->d_x0;
        sa.X = (int)h->X;
        if (h->tdiag)
            for (int64_t c = 0; c < h->C && c < FR_C; c++) sa.tdv[c] = h->T[(size_t)(c * h->C + c)];
        if (!ahead) HIP_TRY(launch_sample(sa, h->tdiag, h->stream));
    }
    // timing level 1 with the cooperative kernel: the rollout launch records its own events
    const bool ev_in_launch = h->timing == 1 && h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK;
    // the rollout launch's event pair: the ring's next pair at level 1, ev[1] / ev_dyn at level 2
    hipEvent_t ev_r0 = h->ev[1], ev_r1 = h->ev_dyn;
    if (h->timing == 1) {
        ev_r0 = h->ev_ring[2 * h->ring_head];
        ev_r1 = h->ev_ring[2 * h->ring_head + 1];
        h->ring_head = (h->ring_head + 1) % mppi_handle::EV_RING;
        h->ring_count = std::min(h->ring_count + 1, (int)mppi_handle::EV_RING);
        h->ring_unread = true;
    }
    if (h->timing >= 1 && !ev_in_launch) HIP_TRY(hipEventRecord(ev_r0, h->stream));
    if (h->dyn_kind == MPPI_DYNAMICS_FRANKARIDGEBACK) {
        FrRolloutArgs a{};
        a.model = h->d_model;
        a.cost = h->d_cost;
        a.table = h->d_table;
        a.steps = h->d_steps;
        a.x0 = h->d_x0;
        a.Ushift = h->d_Us;
        a.noise = h->d_noise;
        a.cost_out = rollout_costs_out(h);
        a.begin = h->begin;
        a.count = h->count;
        a.Rpad = h->Rpad;
        a.dt = h->dt;
        a.H = (int)h->H;
        a.optimal = 0;
        a.status = h->d_status;
        a.cost_kind = h->cost_kind;
        a.energy = h->cost_kind == MPPI_COST_ASSISTED_MANIPULATION && h->am.enable_energy_limit;
        a.trace = h->d_trace;
        a.rec = h->d_rec;
        a.rx = h->d_rx;
        a.rtoken = ++h->relay_token ? h->relay_token : ++h->relay_token;   // (never 0)
        // sharded: this rank's wait timeouts into cost slot R, which the all-reduce carries to every rank
        a.wait_sum = h->comm ? h->d_costs_local + h->R : (sharded(h) ? h->d_costs + h->R : nullptr);
        if (h->debug_updates > 0) {   // mppi_debug_inject: this update's launch carries the fault
            a.debug = h->debug_flags;
            h->debug_updates--;
        }
        if (ahead) {   // U*_shifted read from U* with the shift; the state from the launch
            a.drawn_ahead = 1;
            a.samp = sa;
            a.Ushift = sp.shift_by > 0 ? h->d_U : h->d_Us;
            a.ush = sp.shift_by > 0 ? (int)std::min<int64_t>(sp.shift_by, h->H) : 0;
        }
        // a pending filter() not folded here stays pending: this update's phase 3 supersedes it,
        // and only the latest one is observable (mppi_optimal_cost / logger)
        const bool fold = h->opt_state == mppi_handle::OPT_PENDING;
        if (fold) {   // the previous update's filter() as one more row of the remainder launch
            a.fx0 = h->d_x0_opt;
            a.fU = h->d_U;
            a.fsteps = h->opt_steps;
            a.fcost = h->d_opt;
            a.frec = h->d_rec_opt;
        }
        bool folded = false, costs_done = false, tail = false;
        CoopTail ct;
        a.stats = cost_stats_used(h) ? h->d_cstats : nullptr;
        // the next update's draws in the launch's tail, into the buffer it will write (phase 3 makes
        // the rest with the rank); needs the draws made ahead and no tail switch-off
        a.ahead_noise = (ahead && !tail_draws_disabled(h)) ? h->d_noise_prev : nullptr;
        HIP_TRY(launch_fr_coop_update(a, h->env, h->stream, ev_in_launch ? ev_r0 : nullptr, ev_in_launch ? ev_r1 : nullptr,
                                      &folded, &costs_done, &tail, &h->gargs.roll, &h->gargs.x_kernel, h->graph_dry, &ct,
                                      &h->gargs.roll2));
        h->gargs.folded = folded;
        h->gargs.nroll = ct.launches;
        if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev_dyn, h->stream));
        if (!folded) a.fcost = nullptr;
        // fr_coop_x_kernel (the rows left over, the split) writes 768-B records, fr_coop_kernel compact ones
        if (!costs_done && !h->graph_dry) HIP_TRY(launch_fr_step_cost(cost_args(h, a, !h->gargs.x_kernel), h->stream));
        h->tail_drawn = tail;
        h->info[MPPI_INFO_COOPERATIVE] = 1;
        h->info[MPPI_INFO_FOLDED_FILTER] = folded ? 1 : 0;
        h->info[MPPI_INFO_OBJECTIVE_IN_LAUNCH] = costs_done ? 1 : 0;
        h->info[MPPI_INFO_TAIL_DRAWS] = tail ? 1 : 0;
        h->info[MPPI_INFO_SAMPLING] = ahead ? 2 : 0;
        h->info[MPPI_INFO_ROWS] = h->count + (folded ? 1 : 0);
        h->info[MPPI_INFO_HANDOVER] = h->gargs.x_kernel ? -2 : -1;   // -2: read from the device on request
        if (tail) {   // the rows the launch left to rank_draw_kernel (fr_coop.hip relay_stage, group_draws)
            h->tail_row0 = ct.row0;
            h->tail_xbase = ct.xbase;
            h->tail_nxb = ct.nxb;
        }
        if (folded) h->opt_rec_compact = false;   // the folded row: fr_coop_x_kernel's 768-B records
        if (folded) {   // the optimal cost is ready with this update's rollouts; phase 3's host block
                        // carries it back (finish_kernel copies d_opt), on the same stream
            h->kernel_ms[3] = 0.0f;   // timed inside the rollout launch
            h->opt_state = mppi_handle::OPT_FOLDED;
        }
    } else {
        PmRolloutArgs a{};
        a.pm = h->d_pm;
        a.steps = h->d_steps;
        a.x0 = h->d_x0;
        a.Ushift = h->d_Us;
        a.noise = h->d_noise;
        a.cost_out = rollout_costs_out(h);
        a.begin = h->begin;
        a.count = h->count;
        a.Rpad = h->Rpad;
        a.dt = h->dt;
        a.H = (int)h->H;
        a.optimal = 0;
        HIP_TRY(launch_pm_rollout(a, h->stream));
        if (h->timing >= 1) HIP_TRY(hipEventRecord(ev_r1, h->stream));
    }
    if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev[2], h->stream));
    if (h->host_trace) {
        h->ht_sum[2] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h->t_start).count();
        h->ht_n[2]++;
    }
    h->updated_once = true;
    h->phase_open = true;
    return MPPI_OK;
}

static FinishArgs finish_args(mppi_handle *h)
{
    FinishArgs f{};
    f.status = h->d_status;
    f.status_w = h->d_status;
    f.gsplit = h->d_gsplit;
    f.ns = sharded(h) ? 0 : GRAD_SPLIT;
    f.gpart = h->d_gpart;
    f.gradient = h->d_grad;
    f.Ushift = h->d_Us;
    f.cmin = h->d_cmin;
    f.cmax = h->d_cmax;
    f.gradient_step = h->gradient_step;
    f.control_bound = h->control_bound;
    f.H = (int)h->H;
    f.C = (int)h->C;
    f.t0 = h->rollout_time;
    f.dt = h->dt;
    f.sg_window = h->sg_window;
    f.sg_weights = h->d_sg_w;
    f.sg_uu = h->d_sg_uu;
    f.sg_tt = h->d_sg_tt;
    f.sg_start = h->d_sg_start;
    f.sg_last_trim = h->d_sg_last;
    f.U = h->d_U;
    f.opt_cost = h->d_opt;
    f.out = h->h_out_dev;   // the host block, written in place (no copy launch behind the finish)
    f.seq = (double)(h->publish_seq + 1);   // != 0: the block's flag starts at 0
    f.x0 = h->d_x0;
    f.x0_opt = h->d_x0_opt;
    f.X = (int)h->X;
    f.rank_zero = h->d_rank;
    f.rank_n = h->S <= RANK_TILED_MAX ? h->R : 0;
    f.stats_reset = h->d_cstats;
    f.wait_all = sharded(h) ? h->d_costs + h->R : nullptr;   // (phase-split callers: cleared by phase 1)
    f.wait_local = h->comm ? h->d_costs_local + h->R : nullptr;
    return f;
}

static WGradArgs wgrad_args(const mppi_handle *h)
{
    WGradArgs w{};
    w.cost = h->d_costs;
    w.R = h->R;
    w.cost_scale = h->cost_scale;
    w.status = h->d_status;
    w.noise = h->d_noise;
    w.begin = h->begin;
    w.count = h->count;
    w.Rpad = h->Rpad;
    w.H = (int)h->H;
    w.C = (int)h->C;
    w.gsplit = h->d_gsplit;
    w.wexp = h->d_wexp;
    w.wpart = h->d_wpart;
    w.stats = cost_stats_used(h) ? h->d_cstats : nullptr;
    return w;
}

mppi_status mppi_update_phase2(mppi_handle *h)
{
    if (!h || !h->phase_open) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    WGradArgs w{};
    w.cost = h->d_costs;
    w.R = h->R;
    w.cost_scale = h->cost_scale;
    w.status = h->d_status;
    w.noise = h->d_noise;
    w.begin = h->begin;
    w.count = h->count;
    w.Rpad = h->Rpad;
    w.H = (int)h->H;
    w.C = (int)h->C;
    w.gsplit = h->d_gsplit;
    w.wexp = h->d_wexp;
    w.wpart = h->d_wpart;
    w.stats = cost_stats_used(h) ? h->d_cstats : nullptr;
    h->gargs.wg = w;
    if (h->graph_dry) return MPPI_OK;
    // sharded: the partial gradient is summed here and all-reduced before phase 3
    HIP_TRY(launch_weights_gradient(w, h->d_gpart, sharded(h), h->stream));
    if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev_wg, h->stream));
    return MPPI_OK;
}

// Phase 3's launches (finish, filter() bookkeeping, rank + draws ahead); *seq: the sequence the
// finish kernel publishes.  With graph_dry the arguments go to gargs and nothing is launched.
static mppi_status phase3_launch(mppi_handle *h, double *seq_out)
{
    // the previous update's optimal rollout reads d_U / d_x0_opt: wait for it before rewriting
    if (h->opt_state == mppi_handle::OPT_LAUNCHED) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_opt_done, 0));
    h->gargs.fin = finish_args(h);
    if (!h->graph_dry) HIP_TRY(launch_finish(h->gargs.fin, h->stream));
    const double seq = (double)(++h->publish_seq);
    *seq_out = seq;
    if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev[3], h->stream));
    const bool standalone_filter = h->dyn_kind != MPPI_DYNAMICS_FRANKARIDGEBACK;
    if (standalone_filter) HIP_TRY(hipEventRecord(h->ev_pub, h->stream));   // the side stream waits on it
    // filter(): cost of the published U* (mppi.cpp:450-479).  With the cooperative kernel it rides
    // in the next update's remainder launch (it then shares a SIMD with rollouts 0 and 1 instead of
    // doubling up a SIMD of the next update's main launch); otherwise it runs now on the side stream.
    h->opt_steps = h->d_steps;
    h->opt_state = mppi_handle::OPT_PENDING;
    if (standalone_filter) {
        mppi_status st = launch_filter_standalone(h);
        if (st != MPPI_OK) return st;
    }
    if (h->timing >= 2) HIP_TRY(hipEventRecord(h->ev[5], h->stream));
    // sample()'s stable order of this update's costs (final here: all-reduced when sharded), for
    // the next update.  On the engine stream behind the published block, it runs while the host
    // takes the result and comes back with the next state.
    if (!draw_ahead_possible(h)) HIP_TRY(launch_rank(h->d_costs, h->S, h->d_rank, h->d_rank_keys, h->stream));
    else {   // the next update's draws, into the buffer it will write, with the rank in one launch
        SampleArgs sa{};
        sa.Uprev = h->d_U;
        sa.noise = h->d_noise_prev;
        sa.sp.update_index = h->update_count + 1;
        sa.sp.seed = h->seed;
        sa.begin = h->begin;
        sa.count = h->count;
        sa.Rpad = h->Rpad;
        sa.H = (int)h->H;
        sa.C = (int)h->C;
        for (int64_t c = 0; c < h->C && c < FR_C; c++) sa.tdv[c] = h->T[(size_t)(c * h->C + c)];
        if (h->tail_drawn)
            HIP_TRY(launch_draw_ahead(sa, h->d_costs, h->S, h->d_rank, h->d_rank_keys, h->stream, h->tail_nxb, h->tail_xbase,
                                      h->tail_row0, &h->gargs.rd, h->graph_dry));
        else HIP_TRY(launch_draw_ahead(sa, h->d_costs, h->S, h->d_rank, h->d_rank_keys, h->stream, 0, 0, 0, &h->gargs.rd,
                                       h->graph_dry));
        h->ahead = {h->update_count + 1, h->seed, h->begin, h->count, h->H, h->C};
        h->ahead_valid = true;
    }
    return MPPI_OK;
}

// Phase 3's wait for the published block (sequence `seq`) and the host's bookkeeping.
static mppi_status phase3_wait(mppi_handle *h, double seq)
{
    const int HC = (int)(h->H * h->C);
    // wait for the published block by polling its sequence flag (finish kernels, publish_block): a
    // blocking synchronize sleeps the thread and the wake-up sat on the update's critical path, and
    // an event behind the finish kernel delayed the stream.  The stream is queried now and then so
    // that a failed launch ends the wait with its error, and the wait is bounded: a kernel that
    // never finishes leaves the stream NotReady for good, so past max(5 s, 100 x the last update)
    // the update fails with MPPI_ERR_DEVICE instead of spinning forever.
    {
        volatile double *flag = h->h_out + HC + 6;
        const auto t_wait = std::chrono::steady_clock::now();
        const double limit_s = std::max(h->publish_timeout_s, 100.0 * h->update_duration);
        for (uint64_t spin = 1; *flag != seq; spin++) {
            if ((spin & 4095) == 0) {
                const hipError_t q = hipStreamQuery(h->stream);
                if (q != hipErrorNotReady && q != hipSuccess) HIP_TRY(q);
                if (q == hipSuccess && *flag != seq) return fail(h, MPPI_ERR_DEVICE, "finish kernel did not publish");
                if (q == hipErrorNotReady &&
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t_wait).count() > limit_s) {
                    h->phase_open = false;
                    return fail(h, MPPI_ERR_DEVICE, "update did not publish within " + std::to_string(limit_s) +
                                                        " s (device hung?)");
                }
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (h->host_trace) h->ht_flag = std::chrono::steady_clock::now();
    }
    if (h->timing >= 2) HIP_TRY(hipEventSynchronize(h->ev[5]));
    h->phase_open = false;
    if (h->timing >= 2) {
        for (int i = 0; i < 3; i++) (void)hipEventElapsedTime(&h->kernel_ms[i], h->ev[i], h->ev[i + 1]);
        (void)hipEventElapsedTime(&h->kernel_ms[4], h->ev[0], h->ev[5]);
    }
    if (h->timing >= 2) {
        (void)hipEventElapsedTime(&h->kernel_ms[5], h->ev[1], h->ev_dyn);
        // the weight reduce alone: behind the cost all-reduce when the engine runs it (ev_ar)
        const bool ar = h->comm != nullptr;
        (void)hipEventElapsedTime(&h->kernel_ms[6], ar ? h->ev_ar : h->ev[2], h->ev_wg);
        h->kernel_ms[7] = 0.0f;
        if (ar) (void)hipEventElapsedTime(&h->kernel_ms[7], h->ev[2], h->ev_ar);
    }
    const bool all_nan = h->h_out[HC + 1] != 0.0;
    const bool sg_error = h->h_out[HC + 3] != 0.0;
    const int64_t waits = (int64_t)h->h_out[HC + 7];   // in-launch waits that gave up (the finish kernel)
    h->info[MPPI_INFO_WAIT_TIMEOUTS] = waits;
    h->wait_timeouts_total += waits;
    if (waits) return fail(h, MPPI_ERR_DEVICE, "in-launch wait timed out (" + std::to_string(waits) +
                                                   " waits): rollout costs incomplete, U* not published");
    if (all_nan) return fail(h, MPPI_ERR_ALL_NAN, "all nan rollouts");
    if (sg_error) return fail(h, MPPI_ERR_SMOOTHING, "Savitzky-Golay window: time went backwards");
    {
        std::lock_guard<std::mutex> lock(h->mtx);   // publish under lock (mppi.cpp:178-182)
        h->last_rollout_time = h->rollout_time;
        std::memcpy(h->U_host.data(), h->h_out, (size_t)HC * sizeof(double));
    }
    if (h->d_trace) {   // diagnostics: append this update's per-block records
        std::vector<uint32_t> tr((size_t)(4 * ((h->R + 1) / 4 + 40)));
        HIP_TRY(hipMemcpy(tr.data(), h->d_trace, tr.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (FILE *fp = std::fopen(h->trace_path.c_str(), "ab")) {
            std::fwrite(tr.data(), sizeof(uint32_t), tr.size(), fp);
            std::fclose(fp);
        }
    }
    h->update_duration = std::chrono::duration<double>(std::chrono::steady_clock::now() - h->t_start).count();
    h->update_last = h->rollout_time;
    ++h->update_count;
    h->published_once = true;   // a filter() row exists from here on (mppi_optimal_terms)
    if (h->host_trace) {
        h->ht_ret = std::chrono::steady_clock::now();
        h->ht_sum[0] += std::chrono::duration<double, std::micro>(h->ht_ret - h->ht_flag).count();
        h->ht_n[0]++;
    }
    return MPPI_OK;
}

mppi_status mppi_update_phase3(mppi_handle *h)
{
    if (!h || !h->phase_open) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    double seq = 0.0;
    mppi_status st = phase3_launch(h, &seq);
    if (st != MPPI_OK) return st;
    return phase3_wait(h, seq);
}

// The hipGraph path: the steady-state update (FrankaRidgeback on the cooperative kernel, device
// Philox with the draws made ahead, the previous filter() folded into the rollout launch, the
// objective and the next draws in its tail, no device forecast) is the chain rollout(s) -> weights +
// gradient -> finish -> rank + draws ahead, with or without the Savitzky-Golay finish; sharded over
// the engine's RCCL communicator, ncclAllReduce of the costs after the rollouts and of the partial
// gradient before the finish (configs[4]: "8 x MI355X ... hipGraph-captured control step").  It is
// captured from the first such update's launches, RCCL's included; later updates write their
// arguments (the same structs the eager launches take: state and shift by value, the swapped eps
// buffers, the update index, the publish sequence) into the executable graph's kernel nodes and
// launch it once.  Every rank captures at the same update and replays the graph once per update,
// so the collectives stay matched.  Anything else runs the eager launches.
static bool graph_eligible(const mppi_handle *h)
{
    if (!h->graph_mode || h->timing != 0 || h->d_trace || h->host_trace) return false;
    if (sharded(h) && !h->comm) return false;   // the phase-split API: the caller's collectives
    if (!draw_ahead_possible(h) || tail_draws_disabled(h) || !fr_coop_costs_in_launch(h->env)) return false;
    if (h->fc.type != FC_NONE) return false;   // (the device forecast's sampling launch is not a node)
    if (h->opt_state != mppi_handle::OPT_PENDING) return false;   // the previous filter() folds in
    // the launch path the replayed nodes assume: fr_coop_x_kernel with the filter() row folded and
    // the objective in the launch (a rollout count that is a multiple of 16 takes fr_coop_kernel<4>
    // with filter() left pending, a horizon past 128 steps adds the cost kernel)
    if (!fr_coop_update_folds(h->count, (int)h->H, h->env) || h->debug_updates > 0) return false;
    return h->ahead_valid && h->ahead.update_index == h->update_count && h->ahead.seed == h->seed &&
           h->ahead.begin == h->begin && h->ahead.count == h->count && h->ahead.H == h->H && h->ahead.C == h->C;
}

// The captured graph's kernel nodes in stream order (a topological order of the chain), classified
// by kernel function; RCCL's nodes and the kernels with fixed arguments are left as captured
static mppi_status graph_nodes(mppi_handle *h)
{
    size_t n = 0;
    HIP_TRY(hipGraphGetNodes(h->graph, nullptr, &n));
    std::vector<hipGraphNode_t> nodes(n);
    if (n) HIP_TRY(hipGraphGetNodes(h->graph, nodes.data(), &n));
    std::vector<size_t> indeg(n, 0);
    for (size_t i = 0; i < n; i++) HIP_TRY(hipGraphNodeGetDependencies(nodes[i], nullptr, &indeg[i]));
    std::vector<bool> done(n, false);
    h->gnodes.clear();
    int count[5] = {0, 0, 0, 0, 0};
    for (size_t visited = 0; visited < n;) {   // Kahn's order over the dependency counts
        size_t i = 0;
        while (i < n && (done[i] || indeg[i] != 0)) i++;
        if (i == n) return fail(h, MPPI_ERR_DEVICE, "captured update graph has a cycle");
        done[i] = true;
        visited++;
        size_t nd = 0;
        HIP_TRY(hipGraphNodeGetDependentNodes(nodes[i], nullptr, &nd));
        std::vector<hipGraphNode_t> next(nd);
        if (nd) HIP_TRY(hipGraphNodeGetDependentNodes(nodes[i], next.data(), &nd));
        for (hipGraphNode_t d : next)
            for (size_t k = 0; k < n; k++)
                if (nodes[k] == d && indeg[k] > 0) indeg[k]--;
        hipGraphNodeType ty;
        HIP_TRY(hipGraphNodeGetType(nodes[i], &ty));
        if (ty != hipGraphNodeTypeKernel) continue;
        mppi_handle::GraphNode g{nodes[i], GK_OTHER, 0, {}};
        HIP_TRY(hipGraphKernelNodeGetParams(nodes[i], &g.params));
        g.kind = fr_coop_is_update_kernel(g.params.func) ? GK_ROLLOUT : graph_kernel_kind(g.params.func);
        if (g.kind == GK_OTHER) continue;
        g.index = count[g.kind]++;
        h->gnodes.push_back(g);
    }
    // the launches the arguments are kept for: the rollout launch(es), one weights kernel (and the
    // large-R softmin pair ahead of it), one finish, one rank + draws
    if (count[GK_ROLLOUT] != h->gargs.nroll || count[GK_WGRAD] < 1 || count[GK_FINISH] != 1 || count[GK_RANKDRAW] != 1)
        return fail(h, MPPI_ERR_DEVICE, "captured update graph has " + std::to_string(count[GK_ROLLOUT]) + " rollout, " +
                                            std::to_string(count[GK_WGRAD]) + " weights, " + std::to_string(count[GK_FINISH]) +
                                            " finish and " + std::to_string(count[GK_RANKDRAW]) + " rank nodes");
    return MPPI_OK;
}

// The eager path's collectives (mppi_update), captured with the launches
static mppi_status allreduce_costs(mppi_handle *h)
{
    // R costs and slot R, every rank's in-launch wait timeouts (the finish kernels fail the
    // update on all ranks alike when any rank's launch lost rows)
    NCCL_TRY(ncclAllReduce(h->d_costs_local, h->d_costs, (size_t)h->R + 1, ncclDouble, ncclSum, h->comm, h->stream));
    return MPPI_OK;
}
static mppi_status allreduce_gradient(mppi_handle *h)
{
    NCCL_TRY(ncclAllReduce(h->d_gpart, h->d_gpart, (size_t)(h->H * h->C), ncclDouble, ncclSum, h->comm, h->stream));
    return MPPI_OK;
}

// The host-side state one update's phases advance (phase 1: the shift, the swapped eps buffers, the
// draws-ahead signature, the folded filter(); phase 3: the publish sequence, the pending filter(),
// the next draws' signature).  A capture that fails after recording an update restores it and runs
// the same update eagerly.
struct UpdateSnapshot {
    double last_shift_time, rollout_time;
    int64_t shift_by, shifted;
    double *noise, *noise_prev;
    mppi_handle::AheadSig ahead;
    bool ahead_valid;
    int opt_state;
    const StepConst *opt_steps;
    StepConst *steps;
    uint64_t publish_seq;
};
static UpdateSnapshot snapshot_update(const mppi_handle *h)
{
    return {h->last_shift_time, h->rollout_time, h->shift_by, h->shifted, h->d_noise, h->d_noise_prev,
            h->ahead, h->ahead_valid, (int)h->opt_state, h->opt_steps, h->d_steps, h->publish_seq};
}
static void restore_update(mppi_handle *h, const UpdateSnapshot &u)
{
    h->last_shift_time = u.last_shift_time;
    h->rollout_time = u.rollout_time;
    h->shift_by = u.shift_by;
    h->shifted = u.shifted;
    h->d_noise = u.noise;
    h->d_noise_prev = u.noise_prev;
    h->ahead = u.ahead;
    h->ahead_valid = u.ahead_valid;
    h->opt_state = (decltype(h->opt_state))u.opt_state;
    h->opt_steps = u.opt_steps;
    h->d_steps = u.steps;
    h->publish_seq = u.publish_seq;
    h->phase_open = false;
}

static mppi_status update_eager(mppi_handle *h, const double *state, double time);

// Capture failed after this update's launches were recorded (nothing of it ran): drop the graph for
// good and run the same update eagerly from the restored host state.  Sharded over RCCL this keeps
// the collectives matched - the peer ranks replay (or run eagerly) this update's two all-reduces,
// and this rank issues the same two in the same order - instead of leaving them blocked in the first.
static mppi_status graph_capture_failed(mppi_handle *h, const UpdateSnapshot &u, hipGraph_t g, const double *state, double time,
                                        const std::string &why)
{
    if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
    if (g) (void)hipGraphDestroy(g);
    h->graph_exec = nullptr;
    h->graph = nullptr;
    h->gnodes.clear();
    h->graph_mode = 0;   // never again: the eager path from here on
    h->graph_failures++;
    h->graph_error = why;
    restore_update(h, u);
    return update_eager(h, state, time);
}

static mppi_status update_graph(mppi_handle *h, const double *state, double time)
{
    const bool capture = h->graph_exec == nullptr;
    const bool coll = h->comm != nullptr;
    const UpdateSnapshot snap = snapshot_update(h);
    if (capture) HIP_TRY(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    else h->graph_dry = true;
    mppi_status st = mppi_update_phase1(h, state, time);
    if (st == MPPI_OK && coll && capture) st = allreduce_costs(h);
    if (st == MPPI_OK) st = mppi_update_phase2(h);
    if (st == MPPI_OK && coll && capture) st = allreduce_gradient(h);
    double seq = 0.0;
    if (st == MPPI_OK) st = phase3_launch(h, &seq);
    h->graph_dry = false;
    if (capture) {
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(h->stream, &g);
        if (st != MPPI_OK) {   // a phase failed before its launches: as the eager path would
            if (g) (void)hipGraphDestroy(g);
            h->graph_mode = 0;
            return st;
        }
        if (e != hipSuccess)
            return graph_capture_failed(h, snap, g, state, time, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        hipError_t ie = hipGraphInstantiate(&h->graph_exec, g, nullptr, nullptr, 0);
        if (ie == hipSuccess && h->debug_graph_fail > 0) {   // mppi_debug_inject(MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL)
            h->debug_graph_fail--;
            ie = hipErrorOutOfMemory;
        }
        if (ie != hipSuccess) {
            if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
            h->graph_exec = nullptr;
            return graph_capture_failed(h, snap, g, state, time, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
        }
        h->graph = g;
        st = graph_nodes(h);
        if (st != MPPI_OK) {
            // the instantiated graph holds this update as captured (its collectives included): run it
            // once, then drop it - the next updates are eager, with the same collectives in order
            h->graph_error = h->err;
            h->graph_failures++;
            const hipError_t le = hipGraphLaunch(h->graph_exec, h->stream);
            (void)hipGraphExecDestroy(h->graph_exec);
            (void)hipGraphDestroy(h->graph);
            h->graph_exec = nullptr;
            h->graph = nullptr;
            h->gnodes.clear();
            h->graph_mode = 0;
            HIP_TRY(le);
            return phase3_wait(h, seq);
        }
    } else {
        if (st != MPPI_OK) return st;
        if (!h->gargs.x_kernel || !h->gargs.folded) {   // graph_eligible rules this out; never replay a stale chain
            h->graph_mode = 0;
            return fail(h, MPPI_ERR_DEVICE, "graph update took another launch path");
        }
        RankDrawLaunch &rd = h->gargs.rd;
        void *aroll[2][1] = {{&h->gargs.roll}, {&h->gargs.roll2}};
        void *awg[] = {&h->gargs.wg};
        void *afin[] = {&h->gargs.fin};
        void *ard[] = {&rd.cost, &rd.S, &rd.rank, &rd.nr, &rd.a, &rd.nx, &rd.sub_nxb, &rd.sub_xbase, &rd.sub_row0};
        for (const mppi_handle::GraphNode &g : h->gnodes) {
            hipKernelNodeParams p = g.params;
            p.extra = nullptr;
            switch (g.kind) {
            case GK_ROLLOUT: p.kernelParams = aroll[g.index]; break;
            case GK_WGRAD: p.kernelParams = awg; break;
            case GK_FINISH: p.kernelParams = afin; break;
            default: p.kernelParams = ard; p.gridDim = dim3(rd.grid); break;
            }
            HIP_TRY(hipGraphExecKernelNodeSetParams(h->graph_exec, g.node, &p));
        }
    }
    HIP_TRY(hipGraphLaunch(h->graph_exec, h->stream));
    h->graph_updates++;
    return phase3_wait(h, seq);
}

mppi_status mppi_debug_inject(mppi_handle *h, int fault, int updates)
{
    if (!h || fault < 0 || fault > MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL || updates < 0) return MPPI_ERR_INVALID;
    if (fault == MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL) {   // a host-side fault: no launch carries it
        h->debug_graph_fail = updates;
        return MPPI_OK;
    }
    h->debug_flags = fault;
    h->debug_updates = updates;
    return MPPI_OK;
}

mppi_status mppi_debug_folded_cost(mppi_handle *h, double *cost)
{
    if (!h || !cost) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(cost, h->d_opt, sizeof(double), hipMemcpyDeviceToHost));   // no state change
    return MPPI_OK;
}

mppi_status mppi_set_graph(mppi_handle *h, int enable)
{
    if (!h || enable < 0 || enable > 1) return MPPI_ERR_INVALID;
    h->graph_mode = enable;
    return MPPI_OK;
}

mppi_status mppi_graph_updates(mppi_handle *h, int64_t *count)
{
    if (!h || !count) return MPPI_ERR_INVALID;
    *count = h->graph_updates;
    return MPPI_OK;
}

// The point mass in one launch per update (pm_fused.hip): device Philox noise with a diagonal
// transform, unsharded, no smoothing, timing off or level 1 (MPPI_PM_FUSED=0: the five launches)
static bool pm_fused_eligible(const mppi_handle *h)
{
    if (h->env.pm_fused_off) return false;
    return h->dyn_kind == MPPI_DYNAMICS_POINT_MASS && h->d_pm_sync && h->noise_source == MPPI_NOISE_DEVICE_PHILOX &&
           h->tdiag && !sharded(h) && h->sg_window == 0 && h->timing <= 1 && !h->d_trace;
}

static mppi_status update_pm_fused(mppi_handle *h, const double *state, double time)
{
    HIP_TRY(hipSetDevice(h->device));
    h->t_start = std::chrono::steady_clock::now();
    if (h->host_trace && h->ht_n[0] > h->ht_n[1]) {   // (MPPI_HOST_TRACE, as mppi_update_phase1)
        h->ht_sum[1] += std::chrono::duration<double, std::micro>(h->t_start - h->ht_ret).count();
        h->ht_n[1]++;
    }
    h->rollout_time = time;
    h->shift_by = (int64_t)((time - h->last_shift_time) / h->dt);   // sample(): shift by truncation (mppi.cpp:194-201)
    if (h->shift_by > 0) {
        h->last_shift_time = time;
        h->shifted = std::max<int64_t>(0, h->H - h->shift_by);
    }
    PmFusedArgs a{};
    a.pm = h->pm_host;
    a.steps = h->d_steps;
    a.sp.shift_by = h->shift_by;
    a.sp.shifted = h->shift_by > 0 ? h->shifted : h->H;
    a.sp.keep = keep_count(h);
    a.sp.update_index = h->update_count;
    a.sp.seed = h->seed;
    a.sp.tdiag = 1;
    for (int c = 0; c < 3; c++) a.tdv[c] = h->T[(size_t)(c * h->C + c)];
    std::memcpy(a.x0v, state, (size_t)h->X * sizeof(double));
    a.x0_out = h->d_x0;
    a.X = (int)h->X;
    a.H = (int)h->H;
    a.R = h->R;
    a.Rpad = h->Rpad;
    a.dt = h->dt;
    a.rank = h->d_rank;
    // this update's draws were made ahead by the previous launch's tail when nothing they depend on changed
    a.ahead = h->ahead_valid && h->ahead.update_index == h->update_count && h->ahead.seed == h->seed &&
              h->ahead.begin == h->begin && h->ahead.count == h->count && h->ahead.H == h->H && h->ahead.C == h->C;
    h->ahead_valid = false;
    std::swap(h->d_noise, h->d_noise_prev);   // this update's eps into the other buffer
    a.prev = h->d_noise_prev;
    a.noise = h->d_noise;
    a.ahead_noise = h->d_noise_prev;          // free once the kept columns are copied (grid barrier)
    a.cost = h->d_costs;
    a.wexp = h->d_wexp;
    a.stats = h->d_cstats;
    a.status = h->d_status;
    a.gpart = h->d_pm_part;
    a.tpart = h->d_pm_part + (size_t)h->pm_nblocks * (size_t)(h->H * h->C);
    a.bar = h->d_pm_sync;
    a.ticket = h->d_pm_sync + 1;
    a.epoch = h->pm_epoch + 1;   // committed once the launch is queued (the counters then reach it)
    a.nblocks = h->pm_nblocks;
    a.cost_scale = h->cost_scale;
    a.gradient_step = h->gradient_step;
    a.control_bound = h->control_bound;
    a.cmin = h->d_cmin;
    a.cmax = h->d_cmax;
    a.U = h->d_U;
    a.Us = h->d_Us;
    a.gradient = h->d_grad;
    a.out = h->h_out_dev;
    a.seq = (double)(++h->publish_seq);
    a.opt_cost = h->d_opt;
    a.x0_opt = h->d_x0_opt;
    a.stamps = h->d_pm_stamps;
    // the previous update's pending filter() rides in this launch (block 0's second wave, beside
    // its rollouts); this update's stays pending for the next launch, or for a read (wait_optimal)
    a.fold_filter = h->opt_state == mppi_handle::OPT_PENDING ? 1 : 0;
    a.fx0 = h->d_x0_opt;
    // a filter() of the five-launch path still running on the side stream reads d_U / d_x0_opt
    if (h->opt_state == mppi_handle::OPT_LAUNCHED) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_opt_done, 0));
    hipEvent_t ev_r0 = nullptr, ev_r1 = nullptr;
    if (h->timing == 1) {   // the launch's event pair into the ring (mppi_rollout_kernel_times)
        ev_r0 = h->ev_ring[2 * h->ring_head];
        ev_r1 = h->ev_ring[2 * h->ring_head + 1];
        h->ring_head = (h->ring_head + 1) % mppi_handle::EV_RING;
        h->ring_count = std::min(h->ring_count + 1, (int)mppi_handle::EV_RING);
        h->ring_unread = true;
        HIP_TRY(hipEventRecord(ev_r0, h->stream));
    }
    HIP_TRY(launch_pm_update(a, h->stream));
    if (h->host_trace) {
        h->ht_sum[2] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h->t_start).count();
        h->ht_n[2]++;
    }
    h->pm_epoch = a.epoch;
    if (ev_r1) HIP_TRY(hipEventRecord(ev_r1, h->stream));
    // filter() of this update is left pending (as phase 3 leaves the cooperative launch's); the next
    // update's draws are in d_noise_prev
    h->opt_steps = h->d_steps;
    h->opt_state = mppi_handle::OPT_PENDING;
    h->ahead = {h->update_count + 1, h->seed, h->begin, h->count, h->H, h->C};
    h->ahead_valid = true;
    h->info[MPPI_INFO_COOPERATIVE] = 0;
    h->info[MPPI_INFO_FOLDED_FILTER] = a.fold_filter;
    h->info[MPPI_INFO_OBJECTIVE_IN_LAUNCH] = 1;
    h->info[MPPI_INFO_TAIL_DRAWS] = 1;
    h->info[MPPI_INFO_SAMPLING] = a.ahead ? 2 : 1;
    h->info[MPPI_INFO_ROWS] = h->count;
    h->info[MPPI_INFO_HANDOVER] = -1;
    h->info[MPPI_INFO_FUSED_UPDATE] = 1;
    h->updated_once = true;
    h->phase_open = true;
    mppi_status st = phase3_wait(h, a.seq);
    if (h->d_pm_stamps && st == MPPI_OK) {   // diagnostics: each phase's end after the block's entry
        std::vector<uint64_t> sv((size_t)h->pm_nblocks * PM_STAMPS);
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipMemcpy(sv.data(), h->d_pm_stamps, sv.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull;
        for (unsigned b = 0; b < h->pm_nblocks; b++) t0 = std::min(t0, sv[(size_t)b * PM_STAMPS]);
        for (int i = 0; i < PM_STAMPS; i++) {
            uint64_t mx = t0;   // the phase's last block (s_memrealtime: 100 MHz); the finisher's
                                // stamps only in its block (the others stay 0)
            for (unsigned b = 0; b < h->pm_nblocks; b++) mx = std::max(mx, sv[(size_t)b * PM_STAMPS + i]);
            h->pm_stamp_sum[(size_t)i] += (double)(mx - t0) * 0.01;
        }
        h->pm_stamp_n++;
        HIP_TRY(hipMemset(h->d_pm_stamps, 0, sv.size() * sizeof(uint64_t)));
    }
    return st;
}

mppi_status mppi_update(mppi_handle *h, const double *state, double time)
{
    if (h && state && pm_fused_eligible(h)) return update_pm_fused(h, state, time);
    if (h) h->info[MPPI_INFO_FUSED_UPDATE] = 0;
    if (h && state && graph_eligible(h)) return update_graph(h, state, time);
    return update_eager(h, state, time);
}

static mppi_status update_eager(mppi_handle *h, const double *state, double time)
{
    if (h && sharded(h) && !h->comm) return fail(h, MPPI_ERR_COMM, "sharded handle without communicator: use the phase-split API");
    mppi_status st = mppi_update_phase1(h, state, time);
    if (st != MPPI_OK) return st;
    if (sharded(h) && (st = allreduce_costs(h)) != MPPI_OK) return st;
    if (h->comm && h->timing >= 2) HIP_TRY(hipEventRecord(h->ev_ar, h->stream));
    st = mppi_update_phase2(h);
    if (st != MPPI_OK) return st;
    if (sharded(h) && (st = allreduce_gradient(h)) != MPPI_OK) return st;
    return mppi_update_phase3(h);
}

// ---- queries --------------------------------------------------------------------------------

mppi_status mppi_get(mppi_handle *h, double time, double *control)
{
    if (!h || !control) return MPPI_ERR_INVALID;
    std::lock_guard<std::mutex> lock(h->mtx);
    if (time < h->last_rollout_time) return fail(h, MPPI_ERR_TIME, "get() time precedes the last update");
    double t = (time - h->last_rollout_time) / h->dt;
    const int lower = (int)t, upper = lower + 1;
    const int64_t C = h->C;
    if (upper >= h->H) {
        for (int64_t c = 0; c < C; c++)
            control[c] = h->has_default ? h->cdefault[(size_t)c] : h->U_host[(size_t)((h->H - 1) * C + c)];
        return MPPI_OK;
    }
    t -= lower;
    for (int64_t c = 0; c < C; c++)
        control[c] = (1.0 - t) * h->U_host[(size_t)(lower * C + c)] + t * h->U_host[(size_t)(upper * C + c)];
    return MPPI_OK;
}

mppi_status mppi_costs(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMemcpy(out, h->d_costs, (size_t)h->R * sizeof(double), hipMemcpyDeviceToHost));
    return MPPI_OK;
}

mppi_status mppi_weights(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    // the device keeps e_r and the normaliser (weights_gradient_kernel, finish): w_r = e_r / total,
    // IEEE division as on the device.  Before the first update that got past optimise() the
    // weights are the zeros they were created as.
    Status st{};
    HIP_TRY(hipMemcpy(&st, h->d_status, sizeof(Status), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out, h->d_wexp, (size_t)h->R * sizeof(double), hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < h->R; r++) out[r] = st.total != 0.0 ? out[r] / st.total : 0.0;
    return MPPI_OK;
}

mppi_status mppi_gradient(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMemcpy(out, h->d_grad, (size_t)(h->H * h->C) * sizeof(double), hipMemcpyDeviceToHost));
    return MPPI_OK;
}

mppi_status mppi_optimal_control(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    std::lock_guard<std::mutex> lock(h->mtx);
    std::memcpy(out, h->U_host.data(), h->U_host.size() * sizeof(double));
    return MPPI_OK;
}

static mppi_status wait_optimal(mppi_handle *h)
{
    if (h->opt_state == mppi_handle::OPT_PENDING) {
        mppi_status st = launch_filter_standalone(h);
        if (st != MPPI_OK) return st;
    }
    if (h->opt_state == mppi_handle::OPT_FOLDED) {   // read mid-update: it rode in the rollout launch
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipMemcpy(h->h_opt, h->d_opt, sizeof(double), hipMemcpyDeviceToHost));
    }
    if (h->opt_state != mppi_handle::OPT_LAUNCHED && h->opt_state != mppi_handle::OPT_FOLDED) return MPPI_OK;
    HIP_TRY(hipEventSynchronize(h->ev_opt_done));
    if (h->opt_state == mppi_handle::OPT_LAUNCHED) (void)hipEventElapsedTime(&h->kernel_ms[3], h->ev[4], h->ev_opt_end);
    h->opt_cost = h->h_opt[0];
    h->opt_state = mppi_handle::OPT_NONE;
    return MPPI_OK;
}

mppi_status mppi_synchronize(mppi_handle *h)
{
    if (!h) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return wait_optimal(h);
}

mppi_status mppi_optimal_cost(mppi_handle *h, double *cost)
{
    if (!h || !cost) return MPPI_ERR_INVALID;
    mppi_status st = wait_optimal(h);
    if (st != MPPI_OK) return st;
    std::lock_guard<std::mutex> lock(h->mtx);
    *cost = h->opt_cost;
    return MPPI_OK;
}

mppi_status mppi_optimal_terms(mppi_handle *h, double *terms7)
{
    if (!h || !terms7) return MPPI_ERR_INVALID;
    if (h->dyn_kind != MPPI_DYNAMICS_FRANKARIDGEBACK || h->cost_kind != MPPI_COST_ASSISTED_MANIPULATION)
        return fail(h, MPPI_ERR_UNSUPPORTED, "per-term totals: AssistedManipulation on the cooperative kernel only");
    HIP_TRY(hipSetDevice(h->device));
    if (!h->published_once) {   // before the first update that published: reset(0), no filter() row yet
        for (int i = 0; i < 7; i++) terms7[i] = 0.0;
        return MPPI_OK;
    }
    mppi_status st = wait_optimal(h);   // the filter() row's records are then complete
    if (st != MPPI_OK) return st;
    HIP_TRY(launch_fr_terms(h->d_cost, h->opt_steps, h->d_rec_opt, (int)h->H, h->opt_rec_compact, h->d_terms, h->stream_opt));
    HIP_TRY(hipMemcpyAsync(h->h_opt + 1, h->d_terms, 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream_opt));
    HIP_TRY(hipStreamSynchronize(h->stream_opt));
    std::memcpy(terms7, h->h_opt + 1, 7 * sizeof(double));
    return MPPI_OK;
}

mppi_status mppi_argmin(mppi_handle *h, int64_t *rollout)
{
    if (!h || !rollout) return MPPI_ERR_INVALID;
    std::vector<double> c((size_t)h->R);
    mppi_status st = mppi_costs(h, c.data());
    if (st != MPPI_OK) return st;
    int64_t best = -1;
    for (int64_t i = 0; i < h->R; i++) {
        if (std::isnan(c[(size_t)i])) continue;
        if (best < 0 || c[(size_t)i] < c[(size_t)best]) best = i;   // first minimum
    }
    *rollout = best;
    return MPPI_OK;
}

mppi_status mppi_update_last(mppi_handle *h, double *time)
{
    if (!h || !time) return MPPI_ERR_INVALID;
    *time = h->update_last;
    return MPPI_OK;
}

mppi_status mppi_update_duration(mppi_handle *h, double *seconds)
{
    if (!h || !seconds) return MPPI_ERR_INVALID;
    *seconds = h->update_duration;
    return MPPI_OK;
}

mppi_status mppi_noise(mppi_handle *h, double *out)
{
    if (!h || !out) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    const int64_t HC = h->H * h->C;
    std::vector<double> dev((size_t)(HC * h->Rpad));
    HIP_TRY(hipMemcpy(dev.data(), h->d_noise, dev.size() * sizeof(double), hipMemcpyDeviceToHost));
    std::memset(out, 0, (size_t)(h->R * HC) * sizeof(double));
    for (int64_t lr = 0; lr < h->count; lr++) {   // device [H][Rpad][C] -> reference [R][H][C]
        double *o = out + (h->begin + lr) * HC;
        for (int64_t k = 0; k < h->H; k++)
            for (int64_t c = 0; c < h->C; c++) o[k * h->C + c] = dev[(size_t)((k * h->Rpad + lr) * h->C + c)];
    }
    return MPPI_OK;
}

mppi_status mppi_update_info(mppi_handle *h, int64_t *info, int n)
{
    if (!h || !info || n < 0 || n > MPPI_UPDATE_INFO_N) return MPPI_ERR_INVALID;
    if (n > MPPI_INFO_HANDOVER && h->info[MPPI_INFO_HANDOVER] == -2) {   // the last rollout launch's Status word
        int w = -1;
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipMemcpy(&w, &h->d_status->handover, sizeof(w), hipMemcpyDeviceToHost));
        h->info[MPPI_INFO_HANDOVER] = w;
    }
    h->info[MPPI_INFO_WAIT_TIMEOUTS_TOTAL] = h->wait_timeouts_total;
    h->info[MPPI_INFO_GRAPH_UPDATES] = h->graph_updates;
    h->info[MPPI_INFO_GRAPH_FAILURES] = h->graph_failures;
    h->info[MPPI_INFO_UPDATE_COUNT] = (int64_t)h->update_count;
    std::memcpy(info, h->info, (size_t)n * sizeof(int64_t));
    return MPPI_OK;
}

mppi_status mppi_dims(mppi_handle *h, int64_t *R, int64_t *H, int64_t *C, int64_t *X)
{
    if (!h) return MPPI_ERR_INVALID;
    if (R) *R = h->R;
    if (H) *H = h->H;
    if (C) *C = h->C;
    if (X) *X = h->X;
    return MPPI_OK;
}

mppi_status mppi_smoothing_windows(mppi_handle *h, double *uu, double *tt, int64_t *start_idx)
{
    if (!h || !uu || !tt || !start_idx) return MPPI_ERR_INVALID;
    if (h->sg_window <= 0) return fail(h, MPPI_ERR_INVALID, "smoothing disabled");
    HIP_TRY(hipSetDevice(h->device));
    const size_t n = (size_t)(h->C * (h->H + 2 * h->sg_window + 1));
    HIP_TRY(hipMemcpy(uu, h->d_sg_uu, n * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(tt, h->d_sg_tt, n * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(start_idx, h->d_sg_start, (size_t)h->C * sizeof(int64_t), hipMemcpyDeviceToHost));
    return MPPI_OK;
}

mppi_status mppi_kernel_times(mppi_handle *h, float *ms5)
{
    if (!h || !ms5) return MPPI_ERR_INVALID;
    mppi_status st = wait_optimal(h);
    if (st != MPPI_OK) return st;
    std::memcpy(ms5, h->kernel_ms, 5 * sizeof(float));
    return MPPI_OK;
}

mppi_status mppi_kernel_times_nowait(mppi_handle *h, float *ms5)
{
    return mppi_kernel_times_detail(h, ms5, 5);
}

mppi_status mppi_set_timing(mppi_handle *h, int level)
{
    if (!h || level < 0 || level > 2) return MPPI_ERR_INVALID;
    if (level == 1 && !h->ev_ring[0]) {
        HIP_TRY(hipSetDevice(h->device));
        for (auto &e : h->ev_ring) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    }
    h->timing = level;
    if (level == 2) h->ring_unread = false;   // level 2 times [5] itself (ev[1] / ev_dyn), not the ring
    for (float &m : h->kernel_ms) m = 0.0f;
    return MPPI_OK;
}

mppi_status mppi_kernel_times_detail(mppi_handle *h, float *ms, int n)
{
    if (!h || !ms || n < 0 || n > 8) return MPPI_ERR_INVALID;
    if (h->opt_state == mppi_handle::OPT_LAUNCHED && hipEventQuery(h->ev_opt_end) == hipSuccess)
        (void)hipEventElapsedTime(&h->kernel_ms[3], h->ev[4], h->ev_opt_end);
    if (h->ring_unread) {   // level 1: the newest recorded pair
        const int i = (h->ring_head + mppi_handle::EV_RING - 1) % mppi_handle::EV_RING;
        HIP_TRY(hipEventSynchronize(h->ev_ring[2 * i + 1]));
        (void)hipEventElapsedTime(&h->kernel_ms[5], h->ev_ring[2 * i], h->ev_ring[2 * i + 1]);
        h->ring_unread = false;
    }
    std::memcpy(ms, h->kernel_ms, (size_t)n * sizeof(float));
    return MPPI_OK;
}

mppi_status mppi_rollout_kernel_times(mppi_handle *h, float *ms, int capacity, int *count)
{
    if (!h || !count || capacity < 0 || (capacity > 0 && !ms)) return MPPI_ERR_INVALID;
    HIP_TRY(hipSetDevice(h->device));
    const int n = std::min(h->ring_count, capacity);
    for (int j = 0; j < n; j++) {   // oldest first
        const int i = (h->ring_head + mppi_handle::EV_RING - h->ring_count + j) % mppi_handle::EV_RING;
        HIP_TRY(hipEventSynchronize(h->ev_ring[2 * i + 1]));
        HIP_TRY(hipEventElapsedTime(&ms[j], h->ev_ring[2 * i], h->ev_ring[2 * i + 1]));
    }
    *count = n;
    h->ring_count = 0;
    h->ring_unread = false;   // read: a later level-2 kernel_times(detail) keeps its own [5]
    return MPPI_OK;
}

}  // extern "C"
