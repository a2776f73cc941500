// kernels.hpp — launch interface of kernels.hip for the host runtime (engine.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_types.hpp"
#include "../../include/mppi_amd.h"

namespace mppi_eng {

// Device-side outcome of optimise() (mppi.cpp:344-375) and of the smoothing filter.
struct Status {
    int all_nan;     // <= 1 valid rollout: "all nan rollouts" (mppi.cpp:369-370)
    int early;       // max - min < 1e-6 (or all_nan): weights / gradient / U* untouched
    int sg_error;    // SavitzkyGolay window threw (filter.cpp:37-44, 73-82)
    int handover;    // fr_coop_x_kernel: the step relay stage 1 starts at (relay_stage), or -1 without the relay
    // fr_coop_x_kernel: bounded in-launch waits that gave up in this update's rollout launch (some
    // rows' costs were then never written): the finish kernels fail the update on it and reset it
    int wait_timeouts;
    int pad[3];
    double minimum, maximum, total;   // total: the softmin normaliser, summed by the finish kernels
    double tsplit[8];           // its GRAD_SPLIT partial sums (weights_gradient_kernel)
};

// min / max / count of the update's non-NaN costs, accumulated with order-independent atomics on
// order-preserving keys (exact, so deterministic) by whoever evaluates the objective (the rollout
// launch or fr_step_cost_kernel), and read by weights_gradient_kernel instead of a pass over all R
// costs in each of its blocks.  CS_SLOTS slots, one 128-byte line each, spread the atomics: on one
// address 4099 x 3 of them cost ~40 us.  Reset by the finish kernels (a launch boundary before the
// next update's folds).
constexpr int CS_SLOTS = 64;
struct CostStats {
    unsigned long long kmin[CS_SLOTS * 16];
    unsigned long long kmax[CS_SLOTS * 16];
    unsigned int count[CS_SLOTS * 32];
};

constexpr int MAX_X = 32;   // state dimension bound of the by-value state (FrankaRidgeback 31)
static_assert(FR_X <= MAX_X, "state dimension");

// sample(): the eps tensor of this update (mppi.cpp:242-269), one thread per (step, local rollout).
struct SampleArgs {
    const int *rank;          // [R] stable-order rank of rollouts 2..R-1
    const double *Uprev;      // [H][C]  U* of the previous update (rollout 1 = -U*)
    const double *inj;        // injected eps stream [draws][C]
    const double *T;          // [C][C] noise transform (row-major)
    const double *prev;       // [H][Rpad][C] eps of the previous update (kept rollouts shift it)
    double *noise;            // [H][Rpad][C] eps of this update
    double *Us;               // [H][C] U*_shifted, written when shift_by > 0
    SampleParams sp;
    int64_t begin, count, Rpad;
    int H, C;
    // the update's state, passed by value (no host-to-device copy on the update path): block
    // (0, 0) writes it to x0_out for the rollout kernels
    double x0v[MAX_X];
    double *x0_out;
    int X;
    double tdv[FR_C];   // diagonal noise transform by value (tdiag launches: no loads of T)
};

// optimise() and the partial gradient in one launch (kernels.hip weights_gradient_kernel)
struct WGradArgs {
    const double *cost;    // [R], global rollout index
    int64_t R;
    double cost_scale;
    Status *status;
    const double *noise;   // [H][Rpad][C]
    int64_t begin, count, Rpad;
    int H, C;
    double *gsplit;        // [GRAD_SPLIT][H][C]
    double *wexp;          // [R] unnormalised weights e_r (weights = e_r / Status::total)
    double *wpart;         // [4 * 64] scratch: per-chunk min / max / count / sum (R > SM_LARGE_R)
    const CostStats *stats;   // min / max / count from the cost kernel (unsharded), or null: a pass
};

struct FinishArgs {
    const Status *status;
    Status *status_w;
    const double *gsplit;       // [ns][H][C] gradient stage-1 partials (ns > 0: summed here)
    int ns;
    const double *gpart;        // [H][C] summed (all-reduced when sharded) gradient, ns == 0
    double *gradient;
    double *Ushift;
    const double *cmin, *cmax;
    double gradient_step;
    int control_bound;
    int H, C;
    double t0, dt;
    // Savitzky-Golay state (window 0 = disabled)
    int sg_window;
    const double *sg_weights;   // [2w+1]
    double *sg_uu, *sg_tt;      // [C][H + 2w + 1]
    int64_t *sg_start;          // [C]
    double *sg_last_trim;       // [C]
    // publish: U* <- U*_shifted and the host-visible block [U (H*C), optimal cost, status]
    double *U;
    const double *opt_cost;
    double *out;                // host block [HC + 8]: U*, then status words, then the sequence flag
    double seq;                 // written to out[HC + 6] last, system-scope release (host polls it)
    // filter()'s state: the update's x0 copied for the optimal rollout that runs after it
    const double *x0;
    double *x0_opt;
    int X;
    // the next rank launch accumulates into rank[]: zeroed here when it is the tiled kernel
    int *rank_zero;
    int64_t rank_n;
    // the cost statistics, consumed by weights_gradient_kernel ahead of this launch: reset here for
    // the next update's folds (stream-ordered before its rollout launch; may be null)
    CostStats *stats_reset;
    // the update's in-launch wait timeouts: every rank's (the all-reduced cost slot R) when sharded
    // over RCCL, else null (Status::wait_timeouts); wait_local: this rank's slot, reset here
    const double *wait_all;
    double *wait_local;
};

struct FrRolloutArgs {
    const DevModel *model;
    const DevCost *cost;
    const double *table;      // cooperative kernels: the per-body table (launch_fr_body_table)
    const StepConst *steps;   // [H]
    const double *x0;         // [X]
    const double *Ushift;     // [H][C]  U* shifted to this update
    const double *noise;      // [H][Rpad][C] eps of the local rollouts (sample_kernel)
    double *cost_out;         // [R] (global index) or the optimal-cost scalar
    const Status *status;     // optimal mode: skipped when the update failed (no filter())
    int64_t begin, count, Rpad;
    double dt;
    int H;
    int optimal;
    int cost_kind;            // mppi_cost_kind: AssistedManipulation or TrackPoint
    int energy;               // AssistedManipulation enable_energy_limit: the tank's NLE power
    uint32_t *trace;          // diagnostics (COOP_TRACE builds, MPPI_WAVE_TRACE): per block start, end, hw id, xcc
    // filter() of the previous update folded into this launch as one extra row (fr_coop.hip):
    // its state, published U*, step constants and cost output
    const double *fx0, *fU;
    const StepConst *fsteps;
    double *fcost;
    int64_t xbase, xrows;     // fr_coop_x_kernel: the fifth waves' rows [xbase, xbase + xrows)
    // cooperative kernel: per-step records for the cost kernel, [count][H][FR_REC] (rollout-major:
    // one rollout's records are contiguous), and the folded / standalone filter() row's [H][FR_REC]
    double *rec, *frec;
    // U*_shifted row k is Ushift row min(k + ush, H - 1): ush = 0 with U*_shifted itself, the
    // update's shift with U* (draws made ahead)
    int ush;
    // drawn_ahead: the eps tensor holds this update's draws, made behind the previous update
    // (rank_draw_kernel, the previous launch's tail draws); the launch only copies the kept
    // rollouts' columns into it (samp), and x0 comes from samp.x0v.  Block 0 writes U*_shifted and
    // x0 back for the kernels after it.
    int drawn_ahead;
    SampleArgs samp;
    // costs_in_launch (set by launch_fr_coop_update): the waves evaluate the objective of the rows
    // after their horizon loops (fr_coop.hip launch_costs) instead of fr_step_cost_kernel; stats as
    // in FrCostArgs
    int costs_in_launch;
    CostStats *stats;
    // the next update's draws for the main waves' own rows, made in the launch's idle tail into
    // this buffer (fr_coop.hip tail_draws; null: none): rank_draw_kernel then draws only the rest
    double *ahead_noise;
    // fr_coop_x_kernel: the rows left over travel through four relay stages (fr_coop.hip
    // relay_stage; MPPI_HANDOVER=0 keeps them on one wave beside main wave 0)
    int handover;
    // sharded over RCCL: the rank's slot R of the cost vector the engine all-reduces, to which every
    // in-launch wait that gives up adds 1 (so every rank's finish kernel sees any rank's), or null
    double *wait_sum;
    // MPPI_DEBUG_* fault injection (mppi_debug_inject; 0 in production): bit 0, relay stage 1 of
    // the workgroup with rows left over never signals stage 2 (tests the wait-timeout failure)
    int debug;
    // The relay over relay_k workgroups (fr_coop.hip relay_stage): member m of relay group q is
    // workgroup q + RELAY_STRIDE m and runs stages 4 m .. 4 m + 3 over its share of the horizon's
    // chunks; the lanes' state and the rows' partial cost sums cross between members through rx,
    // tagged with this launch's rtoken (nonzero, one per launch).  relay_k = 1: one workgroup.
    struct RelayXfer *rx;
    uint32_t rtoken;
    int relay_k;
};
constexpr int RELAY_K_MAX = 4, RELAY_STRIDE = 8, RELAY_GROUPS_MAX = 4;
// One relay group's hand-offs between consecutive members (m -> m + 1, m < RELAY_K_MAX - 1): the
// 64 lanes' (q, qd, E) and the four rows' partial cost sums, each behind a token on a line of its own
struct RelayXfer {
    double state[RELAY_K_MAX - 1][64 * 3];
    double sums[RELAY_K_MAX - 1][16];
    uint32_t state_tok[RELAY_K_MAX - 1][32];
    uint32_t sums_tok[RELAY_K_MAX - 1][32];
};

// What the objective reads at (step k, rollout): the state x_k the cost is evaluated at and the
// kinematics of the calculate() before it - the "derived record", FR_NREC doubles.
constexpr int FR_NREC = 42;   // 41 used, padded to 16 bytes
constexpr int REC_QQD = 0;    // [2j], [2j + 1]: q_j, qd_j (j < 12)
constexpr int REC_EE = 24;    // EE position (world)
constexpr int REC_AM = 27;    // arm-mount position (world)
constexpr int REC_E = 30;     // energy tank level (enable_energy_limit)
constexpr int REC_VL = 32;    // EE linear frame velocity J v (bodies 0..9)
constexpr int REC_JJ = 35;    // J_a J_a^T (arm joints 3..9), packed 00 01 02 11 12 22
// What the cooperative rollout kernel stores per (rollout, step) - the "stored record", FR_REC
// doubles: the derived record's first 32 doubles as they are, then two planes of one 16-byte slot
// per lane of the row instead of J v and J_a J_a^T: (S_j linear x, y) and (S_j linear z, qd_j) of
// the calculate() the kinematics come from (lanes 12..15 and the fingers' slots unused).  The
// objective forms J v = sum_j S_j qd_j and J_a J_a^T from them (fr_cost_terms.hpp kin_sums) with
// the FMA chains the rollout kernel's lanes used to run on every step (r05: 50 instructions off the
// dynamics chain, the objective's waves doing them in the slots it leaves idle).
constexpr int REC_S01 = 32;   // [32 + 2j], [33 + 2j]: S_j linear x, y (j < 10 read)
constexpr int REC_S2Q = 64;   // [64 + 2j], [65 + 2j]: S_j linear z, the calculate()'s qd_j (j < 10 read)
constexpr int FR_REC = 96;    // 768 B: sixteen records are 96 whole 128-byte lines
// The compact stored record (fr_coop_kernel: the one-wave and four-wave launches whose waves evaluate
// their own rows' objective after their loops, and the standalone filter()): the derived record
// itself - the rows form J v and J_a J_a^T on their own chain (lane m < 9 writes sum m at REC_VL + m)
// - plus a sink for the frame positions of the lanes that own neither the EE nor the arm mount.
// 384 B: half the 768-B record's bytes, written and read back (sixteen records are 48 lines).
// fr_coop_x_kernel keeps the 768-B record: its objective waves run the sums beside the loops.
constexpr int REC_SINK_C = 42;   // slots 42..44: the other lanes' frame positions, read by nobody
constexpr int FR_REC_C = 48;

// The rollout costs from the records (fr_cost.hip): one wave per rollout, one lane per step, the
// step costs summed in step order (the reference's J += cost, mppi.cpp:322-337).
struct FrCostArgs {
    int compact;              // the records are FR_REC_C compact ones (fr_coop_kernel), else FR_REC
    const DevCost *cost;
    const StepConst *steps;   // [H]
    const double *rec;        // [count][H][FR_REC]
    int64_t begin, count;
    double *cost_out;         // [R] (global index begin + row) or the optimal-cost scalar
    const Status *status;
    int H;
    int optimal;
    int cost_kind;
    int energy;
    // filter() row of the previous update (row == count): its records, constants and output
    const double *frec;
    const StepConst *fsteps;
    double *fcost;
    CostStats *stats;         // the update's rollout costs (not filter()'s) folded in, or null
};

struct PmRolloutArgs {
    const DevPointMass *pm;
    const StepConst *steps;
    const double *x0;
    const double *Ushift;
    const double *noise;      // [H][Rpad][3]
    double *cost_out;
    const Status *status;
    int64_t begin, count, Rpad;
    double dt;
    int H;
    int optimal;
};




// stable rank of rollouts 2..S+1 by cost; `sorted` is scratch of rank_scratch(S) keys
// ---- wrench forecast on the device (forecast.hip) --------------------------------------------
constexpr int FC_NONE = -1, FC_LOCF = 0, FC_AVERAGE = 1, FC_KALMAN = 2;   // mppi_forecast_type
constexpr int KMAX = 24;   // Kalman states 6 (order + 1), order <= 3

// Forecast::forecast(t) inputs: LOCF observation / Average mean (value), LOCF validity, Kalman
// interpolation grid and its prediction table [steps + 1][6] in device memory.
struct ForecastArgs {
    int type;
    int steps;
    double value[6];
    double valid_until;
    double last_update, horison, time_step;
    const double *pred;
};

// trajectory_cost's configuration (assisted_manipulation.hpp) for the per-step constants
struct StepParams {
    int assisted_manipulation;
    int has_forecast;
    double target_scale, target_maximum, position_threshold;
    double pos_c, pos_l, pos_q;
    double vel_dropoff, vel_minimum, vel_maximum;
};

// KalmanFilter state (kalman.hpp) of the forecast's filter, row-major KMAX x KMAX
struct DevKalman {
    double F[KMAX * KMAX], P[KMAX * KMAX];
    double x[KMAX], xn[KMAX], meas[KMAX];
};

struct KalmanObserve {
    int n, order, steps;
    int64_t pending;   // update(time) calls since the last observation
    double dt;         // time - m_last_update
    double m[6];
};

hipError_t launch_forecast_steps(const ForecastArgs &f, const StepParams &p, const double *gamma, int H, double t0, double dt,
                                 StepConst *out, hipStream_t s);
hipError_t launch_kalman_observe(DevKalman *kf, double *pred, const KalmanObserve &a, hipStream_t s);
hipError_t launch_forecast_eval(const ForecastArgs &f, double time, double *out, hipStream_t s);

// stable rank of rollouts 2..S+1 by cost: one all-pairs tiled launch up to RANK_TILED_MAX (rank[]
// must be zero: finish_kernel clears it), chunk sort + merge beyond
constexpr int64_t RANK_TILED_MAX = 8192;
hipError_t launch_rank(const double *cost, int64_t S, int *rank, uint64_t *sorted, hipStream_t s);
inline int64_t rank_scratch(int64_t S) { return ((S + 255) / 256) * 256; }
hipError_t launch_sample(const SampleArgs &a, bool tdiag, hipStream_t s);
// The next update's draws before its state, time and stable order exist (FrankaRidgeback, diagonal
// transform, device Philox): rollout 0 zero, rollout 1 = -U*, the rest Philox by (rollout, step);
// with the stable rank of this update's costs (one launch when S <= RANK_TILED_MAX; rank[] cleared)
// sub_nxb > 0: the rollout launch's tail drew the rest, so only the rows it left are drawn - the
// first wave's rows of its first sub_nxb workgroups (sub_row0 + 16 b + i, i < 4: sub_row0 is the
// first row of the launch that carries the rows left over) and [sub_xbase, count).
// The rank_draw_kernel launch's arguments (the hipGraph path updates its node with them).
struct RankDrawLaunch {
    const double *cost;
    int64_t S;
    int *rank;
    unsigned nr, nx;
    SampleArgs a;
    int sub_nxb;
    int64_t sub_xbase, sub_row0;
    unsigned grid;
};
// dry: fill *out and launch nothing (past RANK_TILED_MAX the rank launches ahead of it are left out too)
hipError_t launch_draw_ahead(const SampleArgs &a, const double *cost, int64_t S, int *rank, uint64_t *sorted,
                             hipStream_t s, int sub_nxb = 0, int64_t sub_xbase = 0, int64_t sub_row0 = 0,
                             RankDrawLaunch *out = nullptr, bool dry = false);
hipError_t launch_pm_rollout(const PmRolloutArgs &a, hipStream_t s);
constexpr int GRAD_SPLIT = 8;   // rollout ranges per step in the gradient's first stage
static_assert(GRAD_SPLIT == sizeof(Status::tsplit) / sizeof(double), "normaliser partials");

// sum_splits (sharded): the GRAD_SPLIT partials are summed into gpart for the all-reduce
hipError_t launch_weights_gradient(const WGradArgs &a, double *gpart, bool sum_splits, hipStream_t s);
hipError_t launch_fr_coop(const FrRolloutArgs &a, hipStream_t s);
// whether launch_fr_coop writes compact records (FR_REC_C): every launch but the standalone filter()
// row's (a.optimal), which keeps the 768-B record and the shorter step of a latency-bound row
bool fr_coop_compact(const FrRolloutArgs &a);
// The update's rollouts (fr_coop_x_kernel): one workgroup per CU of four one-SIMD waves of rollouts
// plus a fifth wave for the rows left over (and, when there are some, the previous update's
// filter() as one more row: *folded).  Falls back to launch_fr_coop beyond one round of CUs.
// The update's rollouts (fr_coop.hip): e0 / e1 = optional timing events around the launch.
// *tail_drawn: the launch made the next update's draws for its main waves' rows (a.ahead_noise).
// final (may be null): the arguments the launch used; *x_kernel: it was fr_coop_x_kernel (one round
// of four-wave workgroups with a fifth wave); dry: decide and fill them, launch nothing.
// Rows past one round of workgroups by less than a workgroup's (fr_coop_update_split) run as two
// launches of fr_coop_x_kernel, the first over one round of full groups (its arguments in *final),
// the second over the rest (*final2); *tail (may be null) tells rank_draw_kernel where the second
// launch's rows left for it are.
struct CoopTail {
    int64_t row0 = 0;    // first row of the launch with the rows left over
    int64_t xbase = 0;   // the rows left over start here (launch rows)
    int nxb = 0;         // workgroups of that launch whose first wave's rows rank_draw_kernel draws
    int launches = 1;
};
struct EnvSwitches;
hipError_t launch_fr_coop_update(const FrRolloutArgs &a, const EnvSwitches &env, hipStream_t s, hipEvent_t e0, hipEvent_t e1, bool *folded,
                                 bool *costs_done, bool *tail_drawn, FrRolloutArgs *final = nullptr, bool *x_kernel = nullptr,
                                 bool dry = false, CoopTail *tail = nullptr, FrRolloutArgs *final2 = nullptr);
bool fr_coop_update_fusable(int64_t count, const EnvSwitches &env);
bool fr_coop_update_split(int64_t count, const EnvSwitches &env);   // the two-launch case of launch_fr_coop_update
bool fr_coop_costs_in_launch(const EnvSwitches &env);   // the objective runs in the update launch (MPPI_COSTS_IN_LAUNCH != 0)
// A/B switches from the environment, read once per mppi_create into the handle (tests set them
// before creating a handle): a handle's launch paths never change under it, and no getenv runs on
// the update path (~80 ns each)
struct EnvSwitches {
    bool draw_ahead_off, tail_draws_off, pm_fused_off, costs_in_launch_off, handover_off, split_off, stream_prio_off;
    int relay_k;   // MPPI_RELAY_K: workgroups the rows left over travel through (1..RELAY_K_MAX; 0: the default)
    // the handle's device: its CU count (the rollout launches' rounds of workgroups) and LDS per
    // block (the fused point mass's residency check), set at create for that device - per handle, so
    // that handles created on different devices from several threads never read each other's
    unsigned cus;
    int lds_max;
};
EnvSwitches env_switches_read();
// Whether a pending filter() folds into the update launch of `count` rows with the objective in
// the launch (fr_coop_x_kernel, one launch or the split's two): the hipGraph path's launch shape
bool fr_coop_update_folds(int64_t count, int H, const EnvSwitches &env);
constexpr int FR_BODY_TABLE = 13 * 46;   // doubles of the cooperative kernels' body table (>= LDS_MODEL)
hipError_t launch_fr_body_table(const DevModel *model, const DevCost *cost, double *table, hipStream_t s);
hipError_t launch_finish(const FinishArgs &a, hipStream_t s);
// The kernel nodes of a captured update graph (engine.cpp update_graph) by their kernel function:
// the ones whose arguments change per update (the rollout launches, the weight reduce, the finish,
// the rank + next draws) and the rest (RCCL's, the gradient sum, the O(S log S) rank), which replay
// with their captured arguments
enum GraphKernel : int { GK_OTHER = 0, GK_ROLLOUT = 1, GK_WGRAD = 2, GK_FINISH = 3, GK_RANKDRAW = 4 };
int graph_kernel_kind(const void *func);          // kernels.hip's kernels
bool fr_coop_is_update_kernel(const void *func);  // fr_coop.hip: an fr_coop_x_kernel instantiation

// FrankaRidgeback::PinocchioDynamics as one device-resident object (fr_object.hip): the members of
// pinocchio_dynamics.hpp:380-425 the methods read and write.
struct DevPinocchio {
    double q[FR_NB], v[FR_NB], tau[FR_NB], a[FR_NB];   // m_joint_position / velocity / torque / acceleration
    double energy, power, time, pad0;                  // EnergyTank, m_power, m_time
    double state[MAX_X];                               // m_state (X = 31 used)
    double ee[MPPI_EE_N];                              // m_end_effector_state (mppi_amd.h MPPI_EE_*)
    double am[3], pad1;                                // the arm-mount frame position (the cost's workspace term)
};
enum ObjOp : int { OBJ_SET_STATE = 0, OBJ_STEP = 1, OBJ_FORECAST = 2, OBJ_COST = 3 };
struct ObjArgs {
    int op;
    DevPinocchio *obj;
    const DevModel *model;
    double x[MAX_X];      // set_state / forecast / cost: the state
    double u[FR_C];       // step: the control
    double time, dt;
    int64_t steps;        // forecast
    const double *wrench; // forecast: [steps][6] forecast(t_k), or null (zeros)
    double *out;          // forecast: [steps][MPPI_DF_N]; cost: [8] total + terms
    DevCost cost;         // cost: the objective
    StepConst sc;         // cost: trajectory_cost's constants of the wrench at `time`
};
hipError_t launch_fr_object(const ObjArgs &a, hipStream_t s);
// forecast(t0 + k dt) for k < steps into out[steps][6] (mppi_forecast_table)
hipError_t launch_forecast_table(const ForecastArgs &f, double t0, double dt, int64_t steps, double *out, hipStream_t s);
hipError_t launch_fr_step_cost(const FrCostArgs &a, hipStream_t s);

// One launch per point-mass update (pm_fused.hip): sample, rollouts, optimise, finish, publish,
// filter() and the next update's rank and draws, with one grid barrier.  Device Philox noise with a
// diagonal transform, unsharded, no smoothing.
constexpr int PM_FUSED_THREADS = 256;
constexpr int64_t PM_FUSED_MAX_R = 4096;
constexpr int PM_FUSED_MAX_BLOCKS = 256;          // one per CU: the grid barrier needs them co-resident
// rollouts per block: the fewest of 16, 32, 64 whose grid (at most 256 blocks) and LDS (the
// finisher stages every block's partials) fit, so that the rank and the draws spread over the most
// CUs; 0 when none does
// (every block must be resident at once for the in-launch grid barrier: the handle's device's CUs
// and LDS per block (EnvSwitches::cus, lds_max), and a shape that does not fit takes the five launches)
int pm_fused_rows(int64_t R, int H, unsigned cus, int lds_max);
struct PmFusedArgs {
    DevPointMass pm;
    const StepConst *steps;     // [H] gamma_k
    SampleParams sp;
    double tdv[3];              // diagonal noise transform
    double x0v[8];              // the update's state by value (X = 6)
    double *x0_out;             // [X] the rollout state (block 0)
    int X;
    int H;
    int64_t R, Rpad;
    double dt;
    int *rank;                  // [R] stable order of the previous costs; rewritten for the next update
    const double *prev;         // [H][Rpad][3] the previous update's eps
    double *noise;              // [H][Rpad][3] this update's eps (draws made ahead when `ahead`)
    double *ahead_noise;        // [H][Rpad][3] the next update's draws, or null
    int ahead;
    double *cost;               // [R]
    double *wexp;               // [R] unnormalised weights e_r
    CostStats *stats;
    Status *status;
    double *gpart;              // [nblocks][H C] partial gradients
    double *tpart;              // [nblocks] partial normalisers
    unsigned *bar, *ticket;     // monotonic arrival counters (targets epoch * nblocks)
    unsigned epoch, nblocks;
    double cost_scale, gradient_step;
    int control_bound;
    const double *cmin, *cmax;
    double *U, *Us, *gradient;  // [H][3]
    double *out;                // the mapped host block [H C + 8]
    double seq;                 // its sequence flag value
    double *opt_cost;           // filter()'s cost of the published U*
    double *x0_opt;             // the update's state, for its filter()
    int fold_filter;            // the previous update's filter() is pending: run it in this launch
    const double *fx0;          // its state (x0_opt as the previous launch left it)
    uint64_t *stamps;           // diagnostics (MPPI_PM_STAMPS=1): [nblocks][PM_STAMPS] s_memrealtime, or null
};
// entry, sampled, rolled out (costs folded into the statistics), barrier passed, partials stored,
// ticket taken, staged, (finisher:) stored, published, ranked, end, costs computed
constexpr int PM_STAMPS = 12;
hipError_t launch_pm_update(const PmFusedArgs &a, hipStream_t s);
// AssistedManipulation's seven per-term totals of one rollout from its [H][FR_REC] records
hipError_t launch_fr_terms(const DevCost *cost, const StepConst *steps, const double *rec, int H, bool compact, double *out7,
                           hipStream_t s);


}  // namespace mppi_eng
