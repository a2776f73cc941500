/*
 * mppi_amd.h — C-ABI of the MI355X-native MPPI trajectory engine.
 *
 * Drop-in boundary for the reference's `mppi::Trajectory` (src/controller/mppi.{hpp,cpp}
 * of LuigiVan01/AssistedManipulation).  Every entry point is `extern "C"`, takes plain
 * pointers and sizes, never throws, and returns an `mppi_status`.  The reference symbol each
 * entry point replaces is cited next to it (paths relative to the reference's src/).
 *
 * Layout conventions (identical to the reference, which stores everything column-major with
 * Eigen):
 *   - a control trajectory is C x H, column-major: element (c, k) at [k * C + c];
 *   - the per-rollout noise tensor handed across the ABI is R x (C x H): rollout r, element
 *     (c, k) at [(r * H + k) * C + c]   (mppi.hpp:281 `Rollout::noise`);
 *   - costs and weights are R-vectors indexed by rollout (R = rollouts + 2, mppi.hpp:306).
 * Inside HBM the engine keeps its own layout; the ABI copies convert.
 */
#ifndef MPPI_AMD_H
#define MPPI_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPPI_AMD_ABI_VERSION 5   /* 5: mppi_device_costs_count, MPPI_INFO_GRAPH_*, MPPI_INFO_UPDATE_COUNT */

#define MPPI_MAX_BODIES 16
#define MPPI_MAX_CONTROL 16
#define MPPI_MAX_STATE 48
#define MPPI_FR_JOINTS 12       /* frankaridgeback/dof.hpp:36-61 DoF::JOINTS */
#define MPPI_FR_STATE 31        /* dof.hpp:63 DoF::STATE */
#define MPPI_FR_CONTROL 12      /* dof.hpp:70 DoF::CONTROL */

typedef enum mppi_status {
    MPPI_OK = 0,
    MPPI_ERR_INVALID = 1,        /* Trajectory::create returns nullptr (mppi.cpp:17-69) */
    MPPI_ERR_DEVICE = 2,         /* HIP runtime failure */
    MPPI_ERR_ALL_NAN = 3,        /* optimise() throws "all nan rollouts" (mppi.cpp:369-370) */
    MPPI_ERR_SMOOTHING = 4,      /* SavitzkyGolay window throws (filter.cpp:37-44, 73-82) */
    MPPI_ERR_TIME = 5,           /* get() asserts monotonic time (mppi.cpp:483) */
    MPPI_ERR_COMM = 6,           /* RCCL failure */
    MPPI_ERR_NOISE = 7,          /* injected noise stream too short for this update */
    MPPI_ERR_UNSUPPORTED = 8
} mppi_status;

/* ------------------------------------------------------------------------------------------
 * Configuration — POD mirror of mppi::Configuration (mppi.hpp:181-249), field for field.
 * Optional fields carry a has_* flag.  `threads` is validated (> 0) as the reference does
 * (mppi.cpp:66-69) and otherwise ignored by the device engine.
 * ---------------------------------------------------------------------------------------- */
typedef struct mppi_config {
    const double *initial_state;   /* X doubles */
    int64_t state_dof;             /* X (must match the dynamics) */
    int64_t control_dof;           /* C (must match the dynamics) */
    int64_t rollouts;              /* S */
    int64_t keep_best_rollouts;    /* K */
    double time_step;
    double horison;                /* H = ceil(horison / time_step) (mppi.cpp:85) */
    double gradient_step;
    double cost_scale;
    double cost_discount_factor;
    const double *covariance;      /* C x C, column-major */
    int32_t control_bound;
    const double *control_min;     /* C */
    const double *control_max;     /* C */
    int32_t has_control_default;
    const double *control_default; /* C, may be NULL when !has_control_default */
    int32_t has_smoothing;
    uint32_t smoothing_window;
    uint32_t smoothing_order;
    uint32_t threads;
} mppi_config;

/* ------------------------------------------------------------------------------------------
 * Dynamics descriptors (replace the mppi::Dynamics plugin object, mppi.hpp:30-85).
 * ---------------------------------------------------------------------------------------- */
typedef enum mppi_dynamics_kind {
    MPPI_DYNAMICS_FRANKARIDGEBACK = 1,  /* FrankaRidgeback::PinocchioDynamics (pinocchio_dynamics.cpp) */
    MPPI_DYNAMICS_POINT_MASS = 2        /* build-defined bring-up plugin */
} mppi_dynamics_kind;

typedef enum mppi_joint_type {
    MPPI_JOINT_REVOLUTE = 0,
    MPPI_JOINT_PRISMATIC = 1
} mppi_joint_type;

/* One moving joint + the rigid body it carries, after fixed-joint merging, in Pinocchio's
 * conventions.  Rotations are row-major 3x3. */
typedef struct mppi_body {
    int32_t parent;          /* parent body index, -1 = universe */
    int32_t type;            /* mppi_joint_type */
    double axis[3];          /* joint axis in the joint frame (unit) */
    double rotation[9];      /* joint placement in the parent joint frame */
    double translation[3];
    double mass;
    double lever[3];         /* centre of mass in the joint frame */
    double inertia[6];       /* rotational inertia about the com, joint frame:
                                xx, xy, yy, xz, yz, zz (Pinocchio Symmetric3 order) */
} mppi_body;

typedef struct mppi_frame {
    int32_t parent;          /* body index the frame is rigidly attached to */
    double rotation[9];      /* placement in that body's joint frame */
    double translation[3];
} mppi_frame;

typedef struct mppi_frankaridgeback_desc {
    int32_t nbodies;                         /* 12 */
    mppi_body bodies[MPPI_MAX_BODIES];
    mppi_frame end_effector;                 /* "panda_grasp_joint" (pinocchio_dynamics.hpp:58) */
    mppi_frame arm_mount;                    /* "arm_mount_joint" (dynamics.cpp:26) */
    double gravity[3];                       /* Pinocchio default (0, 0, -9.81) */
} mppi_frankaridgeback_desc;

typedef struct mppi_point_mass_desc {
    double mass;                             /* state (p[3], v[3]), control = force[3] */
} mppi_point_mass_desc;

typedef struct mppi_dynamics_desc {
    int32_t kind;                            /* mppi_dynamics_kind */
    mppi_frankaridgeback_desc frankaridgeback;
    mppi_point_mass_desc point_mass;
} mppi_dynamics_desc;

/* ------------------------------------------------------------------------------------------
 * Cost descriptors (replace the mppi::Cost plugin object, mppi.hpp:93-145).
 * ---------------------------------------------------------------------------------------- */
typedef enum mppi_cost_kind {
    MPPI_COST_ASSISTED_MANIPULATION = 1,     /* objective/assisted_manipulation.{hpp,cpp} */
    MPPI_COST_QUADRATIC = 2,                 /* point-mass bring-up cost */
    MPPI_COST_TRACK_POINT = 3                /* objective/track_point.{hpp,cpp} */
} mppi_cost_kind;

typedef struct mppi_quadratic {              /* QuadraticCost (controller/cost.hpp:10-37) */
    double constant_cost;
    double linear_cost;
    double quadratic_cost;
} mppi_quadratic;

typedef struct mppi_barrier {                /* Left/RightInverseBarrierFunction (cost.hpp:43-99) */
    double bound;                            /* lower_bound (left) or upper_bound (right) */
    double scale;
    double maximum_cost;                     /* default 1e10 */
} mppi_barrier;

/* AssistedManipulation::Configuration (assisted_manipulation.hpp:16-131), field for field. */
typedef struct mppi_assisted_manipulation_desc {
    int32_t enable_joint_limit;
    int32_t enable_self_collision_limit;
    int32_t enable_workspace_limit;
    int32_t enable_energy_limit;
    int32_t enable_velocity_cost;
    int32_t enable_trajectory_cost;
    int32_t enable_manipulability_cost;
    mppi_barrier lower_joint_limit[MPPI_FR_JOINTS];   /* left barriers */
    mppi_barrier upper_joint_limit[MPPI_FR_JOINTS];   /* right barriers */
    mppi_barrier self_collision_limit;                /* left */
    double self_collision_radii[8];
    mppi_barrier workspace_limit_above;               /* left */
    mppi_barrier workspace_limit_infront;             /* left */
    mppi_barrier workspace_limit_reach;               /* right */
    mppi_quadratic workspace_cost_yaw;
    mppi_barrier energy_limit_below;                  /* left */
    mppi_barrier energy_limit_above;                  /* right */
    mppi_quadratic velocity_cost[MPPI_FR_JOINTS];
    double trajectory_target_scale;
    double trajectory_target_maximum;
    mppi_quadratic trajectory_position_cost;
    double trajectory_position_threshold;
    mppi_quadratic trajectory_velocity_cost;
    double trajectory_velocity_minimum;
    double trajectory_velocity_maximum;
    double trajectory_velocity_dropoff;
    mppi_quadratic manipulability_cost;
    /* The reference's Actor hands the dynamics a DynamicsForecast handle (actor.cpp:85-89);
     * without one trajectory_cost() returns 0 (assisted_manipulation.cpp:239-240). */
    int32_t has_forecast;
} mppi_assisted_manipulation_desc;

/* TrackPoint::Configuration (frankaridgeback/objective/track_point.hpp:20-61), field for field.
 * get_cost (track_point.cpp:10-34) = 100 |p_EE - point|^2, + joint_limit_cost (hard-coded limits,
 * track_point.cpp:45-95; the configured joint barriers are not read), + self_collision_cost,
 * + reach_cost; enable_power_limit is never read. */
typedef struct mppi_track_point_desc {
    double point[3];
    int32_t enable_joint_limits;
    int32_t enable_self_collision_avoidance;
    int32_t enable_power_limit;
    int32_t enable_reach_limits;
    mppi_barrier lower_joint_limit[MPPI_FR_JOINTS];   /* left barriers (configuration only) */
    mppi_barrier upper_joint_limit[MPPI_FR_JOINTS];   /* right barriers (configuration only) */
    mppi_barrier self_collision_limit;                /* left */
    double self_collision_radii[8];
    mppi_barrier maximum_reach_limit;                 /* right */
} mppi_track_point_desc;

typedef struct mppi_quadratic_cost_desc {    /* sum_i q_i (p_i - target_i)^2 + r_i u_i^2 */
    double target[3];
    double q[3];
    double r[3];
} mppi_quadratic_cost_desc;

typedef struct mppi_cost_desc {
    int32_t kind;                            /* mppi_cost_kind */
    mppi_assisted_manipulation_desc assisted_manipulation;
    mppi_quadratic_cost_desc quadratic;
    mppi_track_point_desc track_point;
} mppi_cost_desc;

/* ------------------------------------------------------------------------------------------
 * Engine handle.
 * ---------------------------------------------------------------------------------------- */
typedef struct mppi_handle mppi_handle;

typedef enum mppi_noise_source {
    MPPI_NOISE_DEVICE_PHILOX = 0,   /* eps = T z, z ~ N(0,1) from Philox4x32-10 keyed by (seed, draw) */
    MPPI_NOISE_HOST_INJECTED = 1    /* eps columns supplied by mppi_inject_noise, consumed in
                                       the reference's draw order (mppi.cpp:242-262) */
} mppi_noise_source;

typedef enum mppi_index_semantics {
    MPPI_INDEX_WIDE = 0,            /* 64-bit rollout indices (documented deviation, R > 255) */
    MPPI_INDEX_COMPAT_UINT8 = 1     /* reference std::uint8_t indices (mppi.hpp:639,642); R <= 255 */
} mppi_index_semantics;

/* Library identity / build info. */
int mppi_abi_version(void);
const char *mppi_build_info(void);

/* Defaults: the FrankaRidgeback body table generated from robot.urdf
 * (include/mppi_amd_frankaridgeback.h) and AssistedManipulation::DEFAULT_CONFIGURATION
 * (assisted_manipulation.hpp:133-206). */
void mppi_default_frankaridgeback(mppi_frankaridgeback_desc *out);
void mppi_default_assisted_manipulation(mppi_assisted_manipulation_desc *out);
/* TrackPoint::DEFAULT_CONFIGURATION (track_point.hpp:72-107). */
void mppi_default_track_point(mppi_track_point_desc *out);

/* Trajectory::create (mppi.hpp:321-326, mppi.cpp:11-77).  Validation failures return
 * MPPI_ERR_INVALID with the reference's message available from mppi_last_error(NULL).
 * `device` is the HIP device ordinal the handle binds to. */
mppi_status mppi_create(const mppi_config *config, const mppi_dynamics_desc *dynamics,
                        const mppi_cost_desc *cost, int device, mppi_handle **out);
void mppi_destroy(mppi_handle *h);
/* Last error message of a handle (or of the last failed mppi_create when h == NULL). */
const char *mppi_last_error(const mppi_handle *h);

/* Multi-GPU sample sharding.  Rollouts [begin, end) of this rank are the ones
 * mppi_shard_range assigns; rollouts 0 and 1 always live on rank 0.  world == 1 disables it. */
mppi_status mppi_shard_range(int64_t rollout_count, int world, int rank, int64_t *begin,
                             int64_t *end);
/* Unique id for RCCL bootstrap (128 bytes, ncclUniqueId), produced on rank 0 and broadcast by
 * the caller (e.g. torch.distributed) before mppi_comm_init on every rank. */
mppi_status mppi_comm_unique_id(char out[128]);
mppi_status mppi_comm_init(mppi_handle *h, int world, int rank, const char unique_id[128]);
/* The engine communicator as RCCL reports it (ncclCommCount / ncclCommUserRank; 0 and -1 without
 * one), the handle's HIP device and its PCI bus id (hipDeviceGetPCIBusId, len bytes; may be null):
 * bench.py checks that N ranks form one N-rank communicator on N distinct devices. */
mppi_status mppi_comm_info(mppi_handle *h, int *nranks, int *rank, int *device, char *pci_bus_id, int len);
/* Shard without an engine communicator: the caller runs the two all-reduces between the
 * update phases (mppi_update_phase1..3).  Must precede the first update. */
mppi_status mppi_set_shard(mppi_handle *h, int world, int rank);

/* Parity hooks. */
mppi_status mppi_set_noise_source(mppi_handle *h, int source, uint64_t seed);
/* Supply eps columns (C doubles each) for the next update(s); consumed in draw order. */
mppi_status mppi_inject_noise(mppi_handle *h, const double *eps, int64_t columns);
/* Number of eps columns the next update at `time` will draw (K*shift + (S-K)*H). */
mppi_status mppi_noise_draws(mppi_handle *h, double time, int64_t *columns);
mppi_status mppi_set_index_semantics(mppi_handle *h, int semantics);

/* Per-update forecast table: row k = predicted end-effector wrench (fx fy fz tx ty tz) at
 * t0 + k*dt, k < H (KalmanForecast::forecast, forecast.cpp:342-367, sampled on the step grid). */
mppi_status mppi_set_forecast(mppi_handle *h, const double *wrench_Hx6);

/* Device-resident wrench forecast.  Replaces the caller's table: every
 * update samples Forecast::forecast(t0 + k*dt) for k < H on the device (the rollout queries it
 * through DynamicsForecast::get_end_effector_wrench, dynamics.hpp:275-278, in
 * AssistedManipulation::trajectory_cost, assisted_manipulation.cpp:237-290).  The three kinds of
 * Forecast::Configuration (forecast.hpp:377-416):
 *   LOCFForecast     (forecast.hpp:64-140)   the last observation, zero past its horison;
 *   AverageForecast  (forecast.cpp:41-129)   mean of the observations inside the window;
 *   KalmanForecast   (forecast.cpp:131-367, kalman.cpp:103-152)  Euler state-transition Kalman
 *                    filter over the wrench and its derivatives; each observation runs the filter
 *                    update and the horison of predictions in one device kernel. */
typedef enum mppi_forecast_type {
    MPPI_FORECAST_LOCF = 0,
    MPPI_FORECAST_AVERAGE = 1,
    MPPI_FORECAST_KALMAN = 2
} mppi_forecast_type;

#define MPPI_FORECAST_MAX_ORDER 3   /* Kalman states 6 (order + 1) <= 24 */

typedef struct mppi_forecast_config {
    int32_t type;                         /* mppi_forecast_type */
    /* LOCFForecast::Configuration */
    double locf_observation[6];
    double locf_horison;
    /* AverageForecast::Configuration */
    int32_t average_states;               /* 6: the end-effector wrench */
    double average_window;
    /* KalmanForecast::Configuration */
    int32_t kalman_observed_states;       /* 6: KalmanForecast::update works on Vector6d */
    double kalman_time_step;
    double kalman_horison;
    int32_t kalman_order;                 /* <= MPPI_FORECAST_MAX_ORDER */
    double kalman_initial_state[6];
    /* `variance` is read by create_euler_state_transition_covariance_matrix, which ignores
     * it (forecast.cpp:287-296: 1e-8 I), so it is not carried. */
} mppi_forecast_config;

/* Forecast::create (forecast.cpp:6-39) bound to the handle; failures return MPPI_ERR_INVALID
 * with the reference's message.  NULL detaches (back to mppi_set_forecast tables). */
mppi_status mppi_forecast_attach(mppi_handle *h, const mppi_forecast_config *config);
/* DynamicsForecast::observe_wrench -> Forecast::update(measurement, time). */
mppi_status mppi_forecast_observe(mppi_handle *h, const double *wrench6, double time);
/* DynamicsForecast::observe_time -> Forecast::update(time). */
mppi_status mppi_forecast_observe_time(mppi_handle *h, double time);
/* Forecast::forecast(time) (host copy of the device evaluation). */
mppi_status mppi_forecast_get(mppi_handle *h, double time, double *wrench6);
/* Parity hook: the per-step trajectory-cost constants the last update's rollouts read, H rows of
 * (target x y z, target.target, position cost, velocity target, gamma^k, active). */
mppi_status mppi_step_constants(mppi_handle *h, double *out_Hx8);

/* Trajectory::update (mppi.hpp:339, mppi.cpp:154-187): sample, rollout, optimise, filter,
 * publish.  Blocks until the update is complete on the device. */
mppi_status mppi_update(mppi_handle *h, const double *state, double time);

/* hipGraph path of mppi_update (default off; MPPI_GRAPH=1 at create turns it on): the steady-state
 * update's four launches (rollout, weights + gradient, finish, rank + draws ahead) are captured
 * once and replayed as one graph launch with each update's arguments written into its kernel
 * nodes.  Updates outside that configuration run the eager launches.  mppi_graph_updates counts
 * the updates that ran as the graph. */
mppi_status mppi_set_graph(mppi_handle *h, int enable);
mppi_status mppi_graph_updates(mppi_handle *h, int64_t *count);

/* Phase-split update for callers that run the collectives themselves (multi-GPU with an
 * external communicator, or two shards on one device in tests).  Between phase 1 and 2 the
 * caller all-reduces (sum) the R + 1 doubles of mppi_device_costs(h) - the R costs and slot R,
 * the ranks' in-launch wait timeouts, so that every rank fails an update whose costs some rank
 * lost (MPPI_ERR_DEVICE); between phase 2 and 3 it all-reduces (sum) mppi_device_gradient(h).
 * Buffers are fp64 device pointers on mppi_stream(h). */
mppi_status mppi_update_phase1(mppi_handle *h, const double *state, double time);
mppi_status mppi_update_phase2(mppi_handle *h);
mppi_status mppi_update_phase3(mppi_handle *h);
void *mppi_device_costs(mppi_handle *h);     /* R + 1 doubles (the costs, then the wait-timeout count) */
/* The number of doubles of mppi_device_costs the caller all-reduces: R + 1 since ABI version 4 (R
 * before; a caller that reduces only R loses the cross-rank wait-timeout failure).  Integrators
 * check mppi_abi_version() >= 5 and size the all-reduce from this. */
int64_t mppi_device_costs_count(mppi_handle *h);
void *mppi_device_gradient(mppi_handle *h);  /* C*H doubles */
void *mppi_stream(mppi_handle *h);           /* hipStream_t */

/* filter() (the optimal rollout, mppi.cpp:450-479) runs on a side stream overlapped with the
 * next update's sampling and rollouts; mppi_optimal_cost and mppi_kernel_times wait for it,
 * and mppi_synchronize waits for all device work of the handle. */
mppi_status mppi_synchronize(mppi_handle *h);

/* Trajectory::get (mppi.cpp:481-512): thread-safe against a concurrent update(). */
mppi_status mppi_get(mppi_handle *h, double time, double *control);

/* Observables (logger::MPPI::log reads these, logging/mppi.cpp:84-136). Host copies in the
 * reference layouts. */
mppi_status mppi_costs(mppi_handle *h, double *costs_R);
mppi_status mppi_weights(mppi_handle *h, double *weights_R);
mppi_status mppi_gradient(mppi_handle *h, double *gradient_CxH);
mppi_status mppi_optimal_control(mppi_handle *h, double *control_CxH);
mppi_status mppi_optimal_cost(mppi_handle *h, double *cost);
mppi_status mppi_argmin(mppi_handle *h, int64_t *rollout);
/* The optimal rollout's per-term totals: FrankaRidgeback::AssistedManipulation's accumulators after
 * filter() (thread 0's cost, reset at the optimal rollout's start; assisted_manipulation.cpp:24-35,
 * 74-319), which BaseTest reads by downcasting get_optimal_cost() (test/case/base.cpp:140-146) and
 * logger::AssistedManipulation logs (logging/assisted_manipulation.cpp:61-90).  terms7[MPPI_TERM_*];
 * a disabled term is 0.  AssistedManipulation objective only (MPPI_ERR_UNSUPPORTED otherwise). */
#define MPPI_TERM_JOINT_LIMIT 0      /* get_joint_limit_cost()      (.hpp:232-234) */
#define MPPI_TERM_SELF_COLLISION 1   /* get_self_collision_cost()   (.hpp:236-238) */
#define MPPI_TERM_WORKSPACE 2        /* get_workspace_cost()        (.hpp:240-242) */
#define MPPI_TERM_ENERGY_TANK 3      /* get_energy_tank_cost()      (.hpp:244-246) */
#define MPPI_TERM_JOINT_VELOCITY 4   /* get_joint_velocity_cost()   (.hpp:248-250) */
#define MPPI_TERM_TRAJECTORY 5       /* get_trajectory_cost()       (.hpp:252-254) */
#define MPPI_TERM_MANIPULABILITY 6   /* get_manipulability_cost()   (.hpp:256-258) */
mppi_status mppi_optimal_terms(mppi_handle *h, double *terms7);
mppi_status mppi_update_duration(mppi_handle *h, double *seconds);
/* Trajectory::get_update_last (mppi.hpp:381-384): the time of the last successful update, whichever
 * entry made it (mppi_update, the phase-split calls); the count is MPPI_INFO_UPDATE_COUNT. */
mppi_status mppi_update_last(mppi_handle *h, double *time);
mppi_status mppi_noise(mppi_handle *h, double *noise_R_C_H);
mppi_status mppi_dims(mppi_handle *h, int64_t *rollouts_R, int64_t *steps_H,
                      int64_t *control_C, int64_t *state_X);

/* What the last update's rollout launch did (diagnostics for bench / tests; the engine decides it
 * from the device's CU count and the workload): info[i] for i < n (n <= MPPI_UPDATE_INFO_N). */
#define MPPI_INFO_COOPERATIVE 0           /* 1: the 16-lane cooperative kernel (FrankaRidgeback), 0: the point mass */
#define MPPI_INFO_FOLDED_FILTER 1         /* the previous update's filter() rode in the launch */
#define MPPI_INFO_OBJECTIVE_IN_LAUNCH 2   /* the objective ran in the launch (no cost kernel) */
#define MPPI_INFO_TAIL_DRAWS 3            /* the launch drew the next update's eps (main rows) */
#define MPPI_INFO_SAMPLING 4              /* 0 sample kernel, 1 sampled in the launch (point mass), 2 drawn ahead */
#define MPPI_INFO_ROWS 5                  /* rows rolled out (local rollouts + a folded filter()) */
#define MPPI_INFO_HANDOVER 6              /* step at which relay stage 1 took the rows left over
                                             (relay_stage), -1 none; read from the device */
#define MPPI_INFO_WAIT_TIMEOUTS 7         /* in-launch waits that gave up in the last update's
                                             rollout launch (a bug if nonzero: that update then
                                             failed with MPPI_ERR_DEVICE and published nothing) */
#define MPPI_INFO_WAIT_TIMEOUTS_TOTAL 8   /* the same, summed over every update since create */
#define MPPI_INFO_FUSED_UPDATE 9          /* 1: the whole update ran as one launch (point mass,
                                             pm_update_kernel) */
#define MPPI_INFO_GRAPH_UPDATES 10        /* updates since create that ran as the captured hipGraph */
#define MPPI_INFO_GRAPH_FAILURES 11       /* graph captures that failed (that update then ran eagerly,
                                             its collectives matched; the handle stays eager) */
#define MPPI_INFO_UPDATE_COUNT 12         /* successful updates since create (Trajectory::update
                                             calls that published, whichever entry made them) */
#define MPPI_UPDATE_INFO_N 13
mppi_status mppi_update_info(mppi_handle *h, int64_t *info, int n);

/* Fault injection for the failure-detection tests (no reference counterpart; never set in
 * production): the next `updates` rollout launches carry fault bits `fault`.
 * MPPI_DEBUG_RELAY_NO_SIGNAL: relay stage 1 of the workgroup with rows left over never signals
 * stage 2, so the bounded in-launch waits give up and the update must fail (MPPI_ERR_DEVICE). */
#define MPPI_DEBUG_RELAY_NO_SIGNAL 1
/* MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL: the next `updates` hipGraph captures report an instantiation
 * failure after recording the update (host side; no launch carries it): the update must still run,
 * eagerly, with its collectives, and the handle stays on the eager path. */
#define MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL 2
mppi_status mppi_debug_inject(mppi_handle *h, int fault, int updates);
/* The optimal-rollout cost the device holds now, as the last launch left it, without running or
 * waiting for a pending filter() (tests only): after an update whose launch folded the previous
 * update's filter() (MPPI_INFO_FOLDED_FILTER), that filter()'s cost - which mppi_optimal_cost no
 * longer returns, since it answers for the latest update. */
mppi_status mppi_debug_folded_cost(mppi_handle *h, double *cost);

/* Savitzky-Golay window state (SavitzkyGolayFilter::get_windows(), filter.hpp): per control
 * dimension the value and time buffers (C x (H + 2w + 1), row per dimension) and start index. */
mppi_status mppi_smoothing_windows(mppi_handle *h, double *uu, double *tt, int64_t *start_idx);

/* HIP-event timing of the update path: 0 (default) none, 1 the rollout kernel alone (slot [5] of
 * mppi_kernel_times_detail), 2 every slot.  Each event recorded between two kernels delays the
 * second by a few microseconds, so timing is off unless asked for. */
mppi_status mppi_set_timing(mppi_handle *h, int level);
/* Kernel timing of the last update (HIP events on the engine stream, timing level 2), milliseconds:
 * [0] sample/rank, [1] rollout, [2] weight-reduce, [3] optimal rollout, [4] whole update. */
mppi_status mppi_kernel_times(mppi_handle *h, float *ms5);
/* As mppi_kernel_times without waiting for the side stream: [3] is the latest optimal rollout
 * already finished (possibly an earlier update's).  For timing loops that keep filter() overlapped. */
mppi_status mppi_kernel_times_nowait(mppi_handle *h, float *ms5);
/* The first n (<= 8) per-update times of mppi_kernel_times_nowait, where [5] is the rollout
 * (dynamics) kernel alone: [1] spans it and the FrankaRidgeback cost kernel that sums the step
 * costs from its records; [6] (timing level 2) the weights + gradient launch alone, without the
 * finish kernel that [2] also spans (and, sharded over the engine's RCCL communicator, without the
 * cost all-reduce ahead of it); [7] that cost all-reduce (0 otherwise). */
mppi_status mppi_kernel_times_detail(mppi_handle *h, float *ms, int n);
/* The rollout launch's HIP-event times (ms) of every update run at timing level 1 since the last
 * call, oldest first (at most the last 64): *count <- min(recorded, capacity), and the record is
 * cleared.  Reading them after a timed loop keeps the event queries out of it (querying an event
 * pair right behind the publish held the host ~70 us). */
mppi_status mppi_rollout_kernel_times(mppi_handle *h, float *ms, int capacity, int *count);


/* ------------------------------------------------------------------------------------------
 * FrankaRidgeback::PinocchioDynamics as a device object (one trajectory).  The reference's
 * plugin is also an object with its own state (mppi.hpp:47-84, dynamics.hpp:416-537): the Actor's
 * DynamicsForecast steps one forward every controller period (dynamics.cpp:104-138), and a cost
 * reads the dynamics' cached end-effector state.  Its state lives in HBM and each call is one
 * single-thread kernel (pinocchio_dynamics.cpp:142-260 semantics, quirks included: set_state's
 * calculate() adds NLE onto the torque the previous call left).  FrankaRidgeback only.
 * ---------------------------------------------------------------------------------------- */
typedef struct mppi_dynamics mppi_dynamics;

/* EndEffectorState (dynamics.hpp:95-117) of the last calculate(), doubles: */
#define MPPI_EE_POSITION 0               /* 3: oMf[panda_grasp_joint].translation() */
#define MPPI_EE_QUATERNION 3             /* 4: orientation, Eigen coefficient order (x, y, z, w) */
#define MPPI_EE_ROTATION 7               /* 9: the same orientation as a row-major rotation matrix */
#define MPPI_EE_LINEAR_VELOCITY 16       /* 3: getFrameVelocity(WORLD).linear() */
#define MPPI_EE_ANGULAR_VELOCITY 19      /* 3 */
#define MPPI_EE_LINEAR_ACCELERATION 22   /* 3: getFrameAcceleration(WORLD).linear() (no gravity) */
#define MPPI_EE_ANGULAR_ACCELERATION 25  /* 3 */
#define MPPI_EE_JACOBIAN 28              /* 72: 6 x 12 row-major, WORLD, top-left 3x3 = R_z(yaw) */
#define MPPI_EE_N 100

/* One row of DynamicsForecast::forecast per step (dynamics.cpp:113-127), doubles: */
#define MPPI_DF_JOINT_POSITION 0                   /* 12: m_joint_position[step] */
#define MPPI_DF_END_EFFECTOR 12                    /* MPPI_EE_N: m_end_effector[step] */
#define MPPI_DF_JOINT_POWER (12 + MPPI_EE_N)       /* m_joint_power[step] (0 for Pinocchio) */
#define MPPI_DF_EXTERNAL_POWER (13 + MPPI_EE_N)    /* m_external_power[step] (0 for Pinocchio) */
#define MPPI_DF_ENERGY (14 + MPPI_EE_N)            /* m_energy[step]: the tank */
#define MPPI_DF_WRENCH (15 + MPPI_EE_N)            /* 6: m_end_effector_wrench[step] = forecast(t) */
#define MPPI_DF_N (21 + MPPI_EE_N)

/* PinocchioDynamics::create (pinocchio_dynamics.cpp:19-83; the constructor's set_state of the
 * configuration's initial state, :84-115).  `initial_state`: X = 31 doubles. */
mppi_status mppi_dynamics_create(const mppi_dynamics_desc *desc, const double *initial_state, int device,
                                 mppi_dynamics **out);
void mppi_dynamics_destroy(mppi_dynamics *d);
/* set_state (pinocchio_dynamics.cpp:142-151). */
mppi_status mppi_dynamics_set_state(mppi_dynamics *d, const double *state, double time);
/* step (pinocchio_dynamics.cpp:226-260): control C = 12; the new state (X) into state_out (may be NULL). */
mppi_status mppi_dynamics_step(mppi_dynamics *d, const double *control, double dt, double *state_out);
/* get_state (m_state, X doubles). */
mppi_status mppi_dynamics_get_state(mppi_dynamics *d, double *state);
/* get_end_effector_state (MPPI_EE_N doubles). */
mppi_status mppi_dynamics_end_effector(mppi_dynamics *d, double *ee);
/* The object's other members after its last call: joint position, velocity, acceleration,
 * torque (12 each), tank energy, power, time, arm-mount frame position (3) = 54 doubles. */
#define MPPI_DYNAMICS_QUERY_N 54
mppi_status mppi_dynamics_query(mppi_dynamics *d, double *out);
/* DynamicsForecast::forecast(state, time) (dynamics.cpp:104-138): set_state, then `steps` times
 * record the row and step with Control::Zero() over time_step.  `wrench`: steps x 6 rows of
 * forecast(time + k time_step) (e.g. mppi_forecast_table), copied into the rows; NULL: zeros.
 * out: steps x MPPI_DF_N. */
mppi_status mppi_dynamics_forecast(mppi_dynamics *d, const double *state, double time, double time_step,
                                   int64_t steps, const double *wrench, double *out);
/* Cost::get_cost(state, control, dynamics, time) (mppi.hpp:127-132) of AssistedManipulation
 * (assisted_manipulation.cpp:37-72) or TrackPoint (track_point.cpp:10-34) on the device against the
 * object's cached kinematics.  wrench6: forecast(time) of the dynamics' forecast handle, or NULL
 * when it has none (trajectory_cost is then 0, :239-240).  out: the cost, then the seven
 * AssistedManipulation terms (MPPI_TERM_*; zeros for TrackPoint) = 8 doubles. */
mppi_status mppi_cost_evaluate(const mppi_cost_desc *cost, mppi_dynamics *d, const double *state,
                               const double *control, const double *wrench6, double *out8);
/* forecast(t0 + k dt) for k < steps of the handle's attached forecast (steps x 6). */
mppi_status mppi_forecast_table(mppi_handle *h, double t0, double dt, int64_t steps, double *out);

#ifdef __cplusplus
}
#endif

#endif /* MPPI_AMD_H */
