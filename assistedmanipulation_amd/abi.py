"""ctypes mirror of include/mppi_amd.h (the engine's C-ABI structs and enums).

Pure data definitions: no compute.  Field order and types must match the header exactly;
tests/test_abi.py checks sizes against the compiled library.
"""
import ctypes as C

MPPI_MAX_BODIES = 16
MPPI_FR_JOINTS = 12
MPPI_FR_STATE = 31
MPPI_FR_CONTROL = 12

# mppi_status
MPPI_OK = 0
MPPI_ERR_INVALID = 1
MPPI_ERR_DEVICE = 2
MPPI_ERR_ALL_NAN = 3
MPPI_ERR_SMOOTHING = 4
MPPI_ERR_TIME = 5
MPPI_ERR_COMM = 6
MPPI_ERR_NOISE = 7
MPPI_ERR_UNSUPPORTED = 8

STATUS_NAMES = {
    0: "MPPI_OK", 1: "MPPI_ERR_INVALID", 2: "MPPI_ERR_DEVICE", 3: "MPPI_ERR_ALL_NAN",
    4: "MPPI_ERR_SMOOTHING", 5: "MPPI_ERR_TIME", 6: "MPPI_ERR_COMM", 7: "MPPI_ERR_NOISE",
    8: "MPPI_ERR_UNSUPPORTED",
}

MPPI_DYNAMICS_FRANKARIDGEBACK = 1
MPPI_DYNAMICS_POINT_MASS = 2
MPPI_JOINT_REVOLUTE = 0
MPPI_JOINT_PRISMATIC = 1
MPPI_COST_ASSISTED_MANIPULATION = 1
MPPI_COST_QUADRATIC = 2
MPPI_COST_TRACK_POINT = 3
MPPI_NOISE_DEVICE_PHILOX = 0
MPPI_NOISE_HOST_INJECTED = 1
MPPI_INDEX_WIDE = 0
MPPI_INDEX_COMPAT_UINT8 = 1
MPPI_UPDATE_INFO_N = 13   # mppi_update_info slots (MPPI_INFO_*)
MPPI_DEBUG_RELAY_NO_SIGNAL = 1   # mppi_debug_inject: relay stage 1 never signals stage 2
MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL = 2   # mppi_debug_inject: the next graph captures fail to instantiate
# EndEffectorState layout (MPPI_EE_*) and DynamicsForecast rows (MPPI_DF_*)
MPPI_EE_POSITION, MPPI_EE_QUATERNION, MPPI_EE_ROTATION = 0, 3, 7
MPPI_EE_LINEAR_VELOCITY, MPPI_EE_ANGULAR_VELOCITY = 16, 19
MPPI_EE_LINEAR_ACCELERATION, MPPI_EE_ANGULAR_ACCELERATION = 22, 25
MPPI_EE_JACOBIAN, MPPI_EE_N = 28, 100
MPPI_DF_JOINT_POSITION, MPPI_DF_END_EFFECTOR = 0, 12
MPPI_DF_JOINT_POWER, MPPI_DF_EXTERNAL_POWER, MPPI_DF_ENERGY, MPPI_DF_WRENCH = 112, 113, 114, 115
MPPI_DF_N = 121
MPPI_DYNAMICS_QUERY_N = 54
TERM_NAMES = ("joint_limit", "self_collision", "workspace", "energy_tank", "joint_velocity", "trajectory",
              "manipulability")

_d = C.c_double
_dp = C.POINTER(C.c_double)


class mppi_config(C.Structure):
    _fields_ = [
        ("initial_state", _dp),
        ("state_dof", C.c_int64),
        ("control_dof", C.c_int64),
        ("rollouts", C.c_int64),
        ("keep_best_rollouts", C.c_int64),
        ("time_step", _d),
        ("horison", _d),
        ("gradient_step", _d),
        ("cost_scale", _d),
        ("cost_discount_factor", _d),
        ("covariance", _dp),
        ("control_bound", C.c_int32),
        ("control_min", _dp),
        ("control_max", _dp),
        ("has_control_default", C.c_int32),
        ("control_default", _dp),
        ("has_smoothing", C.c_int32),
        ("smoothing_window", C.c_uint32),
        ("smoothing_order", C.c_uint32),
        ("threads", C.c_uint32),
    ]


class mppi_body(C.Structure):
    _fields_ = [
        ("parent", C.c_int32),
        ("type", C.c_int32),
        ("axis", _d * 3),
        ("rotation", _d * 9),
        ("translation", _d * 3),
        ("mass", _d),
        ("lever", _d * 3),
        ("inertia", _d * 6),
    ]


class mppi_frame(C.Structure):
    _fields_ = [("parent", C.c_int32), ("rotation", _d * 9), ("translation", _d * 3)]


class mppi_frankaridgeback_desc(C.Structure):
    _fields_ = [
        ("nbodies", C.c_int32),
        ("bodies", mppi_body * MPPI_MAX_BODIES),
        ("end_effector", mppi_frame),
        ("arm_mount", mppi_frame),
        ("gravity", _d * 3),
    ]


class mppi_point_mass_desc(C.Structure):
    _fields_ = [("mass", _d)]


class mppi_dynamics_desc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("frankaridgeback", mppi_frankaridgeback_desc),
        ("point_mass", mppi_point_mass_desc),
    ]


class mppi_quadratic(C.Structure):
    _fields_ = [("constant_cost", _d), ("linear_cost", _d), ("quadratic_cost", _d)]


class mppi_barrier(C.Structure):
    _fields_ = [("bound", _d), ("scale", _d), ("maximum_cost", _d)]


class mppi_assisted_manipulation_desc(C.Structure):
    _fields_ = [
        ("enable_joint_limit", C.c_int32),
        ("enable_self_collision_limit", C.c_int32),
        ("enable_workspace_limit", C.c_int32),
        ("enable_energy_limit", C.c_int32),
        ("enable_velocity_cost", C.c_int32),
        ("enable_trajectory_cost", C.c_int32),
        ("enable_manipulability_cost", C.c_int32),
        ("lower_joint_limit", mppi_barrier * MPPI_FR_JOINTS),
        ("upper_joint_limit", mppi_barrier * MPPI_FR_JOINTS),
        ("self_collision_limit", mppi_barrier),
        ("self_collision_radii", _d * 8),
        ("workspace_limit_above", mppi_barrier),
        ("workspace_limit_infront", mppi_barrier),
        ("workspace_limit_reach", mppi_barrier),
        ("workspace_cost_yaw", mppi_quadratic),
        ("energy_limit_below", mppi_barrier),
        ("energy_limit_above", mppi_barrier),
        ("velocity_cost", mppi_quadratic * MPPI_FR_JOINTS),
        ("trajectory_target_scale", _d),
        ("trajectory_target_maximum", _d),
        ("trajectory_position_cost", mppi_quadratic),
        ("trajectory_position_threshold", _d),
        ("trajectory_velocity_cost", mppi_quadratic),
        ("trajectory_velocity_minimum", _d),
        ("trajectory_velocity_maximum", _d),
        ("trajectory_velocity_dropoff", _d),
        ("manipulability_cost", mppi_quadratic),
        ("has_forecast", C.c_int32),
    ]


class mppi_quadratic_cost_desc(C.Structure):
    _fields_ = [("target", _d * 3), ("q", _d * 3), ("r", _d * 3)]


class mppi_track_point_desc(C.Structure):
    _fields_ = [
        ("point", _d * 3),
        ("enable_joint_limits", C.c_int32),
        ("enable_self_collision_avoidance", C.c_int32),
        ("enable_power_limit", C.c_int32),
        ("enable_reach_limits", C.c_int32),
        ("lower_joint_limit", mppi_barrier * MPPI_FR_JOINTS),
        ("upper_joint_limit", mppi_barrier * MPPI_FR_JOINTS),
        ("self_collision_limit", mppi_barrier),
        ("self_collision_radii", _d * 8),
        ("maximum_reach_limit", mppi_barrier),
    ]


class mppi_cost_desc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("assisted_manipulation", mppi_assisted_manipulation_desc),
        ("quadratic", mppi_quadratic_cost_desc),
        ("track_point", mppi_track_point_desc),
    ]


def dptr(arr):
    """ctypes double* into a contiguous float64 numpy array (keeps no reference!)."""
    return arr.ctypes.data_as(_dp)


MPPI_FORECAST_LOCF = 0
MPPI_FORECAST_AVERAGE = 1
MPPI_FORECAST_KALMAN = 2
MPPI_FORECAST_MAX_ORDER = 3


class mppi_forecast_config(C.Structure):
    """Forecast::Configuration (controller/forecast.hpp:377-416) -> include/mppi_amd.h."""
    _fields_ = [
        ("type", C.c_int32),
        ("locf_observation", C.c_double * 6),
        ("locf_horison", C.c_double),
        ("average_states", C.c_int32),
        ("average_window", C.c_double),
        ("kalman_observed_states", C.c_int32),
        ("kalman_time_step", C.c_double),
        ("kalman_horison", C.c_double),
        ("kalman_order", C.c_int32),
        ("kalman_initial_state", C.c_double * 6),
    ]
