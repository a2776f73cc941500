// engine_types.hpp — POD blocks shared by the host runtime and the kernels.
//
// The FrankaRidgeback kernel is specialised for the reference robot's kinematic *topology*
// (parents, joint kinds — frankaridgeback/dof.hpp and robot.urdf); every
// numeric model parameter (placements, masses, inertias, frames) is runtime data uploaded from
// the mppi_frankaridgeback_desc.  mppi_create checks the descriptor against the topology.
#pragma once

#include <stdint.h>

namespace mppi_eng {

// ---- FrankaRidgeback topology --------------------------------------------------------------
constexpr int FR_NB = 12;
constexpr int FR_C = 12;
constexpr int FR_X = 31;
enum JointKind : int { KIND_PX = 0, KIND_PY = 1, KIND_RZ = 2, KIND_PNY = 3 };   // PNY: axis (0,-1,0)
constexpr int FR_PARENT[FR_NB] = {-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9};
constexpr int FR_KIND[FR_NB] = {KIND_PX, KIND_PY, KIND_RZ, KIND_RZ, KIND_RZ, KIND_RZ, KIND_RZ,
                                KIND_RZ, KIND_RZ, KIND_RZ, KIND_PY, KIND_PNY};
constexpr int FR_EE_PARENT = 9;   // panda_grasp_joint is on panda_joint7's body
constexpr int FR_AM_PARENT = 2;   // arm_mount_joint is on pivot_joint's body
constexpr int FR_ARM0 = 3, FR_ARM1 = 10;   // arm joints [3, 10): Jacobian columns of the cost

struct DevBody {
    double R[9];     // placement rotation (row-major) in the parent joint frame
    double p[3];
    double mass;
    double c[3];     // com in the joint frame
    double Ic[6];    // xx, xy, yy, xz, yz, zz about the com
};

struct DevModel {
    DevBody b[FR_NB];
    double ee_R[9], ee_p[3];
    double am_R[9], am_p[3];
    // placement of body 11 relative to body 10's placement, (R10^T R11, R10^T (p11 - p10)): the
    // cooperative kernel's prefix scan reaches finger 11 through finger 10 (fr_coop.hip)
    double f11_R[9], f11_p[3];
    double gravity[3];   // Pinocchio's model.gravity: the NLE of the energy tank's power
};

struct DevBarrier {
    double bound, scale, max;
};

// AssistedManipulation parameters in device form.  Per-step forecast-derived constants live in
// StepConst; the self-collision term is a per-step constant for PinocchioDynamics (link
// positions are the zero stub, pinocchio_dynamics.hpp:189-192) and is folded on the host.
struct DevCost {
    int en_joint, en_self, en_work, en_energy, en_vel, en_traj, en_manip, pad0;
    DevBarrier lower[FR_NB], upper[FR_NB];
    double self_collision;   // sum over the 20 pairs, evaluated on the host in fp64
    DevBarrier ws_above, ws_infront, ws_reach;
    double yaw_c, yaw_l, yaw_q;
    double vel_q[FR_NB];
    double manip_c, manip_l, manip_q;
    double traj_vel_c, traj_vel_l, traj_vel_q;
    // TrackPoint (frankaridgeback/objective/track_point.cpp) when kind == MPPI_COST_TRACK_POINT
    int kind, tp_en_joint, tp_en_self, tp_en_reach;
    double tp_point[3];
    double tp_lo[FR_NB], tp_up[FR_NB];   // joint_limit_cost's hard-coded limits (joints 0..9 read)
    double tp_self;                      // self_collision_cost with get_link_position == 0
    DevBarrier tp_reach;                 // maximum_reach_limit (right)
    // energy_cost (assisted_manipulation.cpp:211-222): Left / Right barriers of the tank energy
    DevBarrier en_below, en_above;
};

// trajectory_cost() constants of step k (assisted_manipulation.cpp:237-290): everything that
// depends only on the forecast wrench at t0 + k dt.
struct StepConst {
    double target[3];
    double tt;          // target . target
    double pos_cost;    // trajectory_position_cost(distance)
    double vtarget;     // clamp(exp(dropoff * distance) - 1, vmin, vmax)
    double gamma_k;     // pow(cost_discount_factor, k)
    int active;         // has forecast && distance > threshold
    int pad;
};

// Quadratic point-mass plugin.
struct DevPointMass {
    double inv_mass;
    double target[3], q[3], r[3];
};

// Per-update sampling parameters (Trajectory::sample, mppi.cpp:189-270).
struct SampleParams {
    int64_t shift_by;     // steps shifted this update (<= 0: no shift)
    int64_t shifted;      // columns kept from the previous noise: H - min(shift_by, H)
    int64_t keep;         // number of kept rollouts K
    int64_t keep_draws;   // draws consumed by kept rollouts' tails: K * min(shift_by, H) or 0
    uint64_t update_index;
    uint64_t seed;
    int injected;         // 1: eps from the injected stream, 0: Philox
    int tdiag;            // 1: noise transform is diagonal
};

}  // namespace mppi_eng
