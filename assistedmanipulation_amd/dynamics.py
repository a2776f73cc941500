"""FrankaRidgeback::PinocchioDynamics as a device object, and DynamicsForecast on top of it.

The reference's plugins are objects with their own state, used outside mppi::Trajectory too:
PinocchioDynamics has set_state / step / get_state / get_end_effector_state
(frankaridgeback/pinocchio_dynamics.{hpp,cpp}, the mppi::Dynamics surface of mppi.hpp:47-84), and
the Actor's DynamicsForecast rolls its own copy forward with zero control every controller period
(frankaridgeback/dynamics.cpp:104-138, actor.cpp:176-177).  Here the object's state lives in HBM
and every method is a device kernel (fr_object.hip, through mppi_dynamics_* of the C-ABI); the
host keeps only the bookkeeping the reference keeps on the caller's side (DynamicsForecast's
trajectories and its time parameterisation, dynamics.hpp:243-345).
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi
from ._lib import load


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


@dataclass
class EndEffectorState:
    """EndEffectorState (dynamics.hpp:95-117) of a calculate()."""
    position: np.ndarray
    orientation: np.ndarray          # quaternion, Eigen coefficient order (x, y, z, w)
    rotation: np.ndarray             # the same orientation, 3 x 3
    linear_velocity: np.ndarray
    angular_velocity: np.ndarray
    linear_acceleration: np.ndarray
    angular_acceleration: np.ndarray
    jacobian: np.ndarray             # 6 x 12, WORLD

    @staticmethod
    def from_row(r):
        r = np.asarray(r, dtype=np.float64)
        return EndEffectorState(
            position=r[abi.MPPI_EE_POSITION:abi.MPPI_EE_POSITION + 3].copy(),
            orientation=r[abi.MPPI_EE_QUATERNION:abi.MPPI_EE_QUATERNION + 4].copy(),
            rotation=r[abi.MPPI_EE_ROTATION:abi.MPPI_EE_ROTATION + 9].reshape(3, 3).copy(),
            linear_velocity=r[abi.MPPI_EE_LINEAR_VELOCITY:abi.MPPI_EE_LINEAR_VELOCITY + 3].copy(),
            angular_velocity=r[abi.MPPI_EE_ANGULAR_VELOCITY:abi.MPPI_EE_ANGULAR_VELOCITY + 3].copy(),
            linear_acceleration=r[abi.MPPI_EE_LINEAR_ACCELERATION:abi.MPPI_EE_LINEAR_ACCELERATION + 3].copy(),
            angular_acceleration=r[abi.MPPI_EE_ANGULAR_ACCELERATION:abi.MPPI_EE_ANGULAR_ACCELERATION + 3].copy(),
            jacobian=r[abi.MPPI_EE_JACOBIAN:abi.MPPI_EE_JACOBIAN + 72].reshape(6, 12).copy())


class PinocchioDynamicsObject:
    """FrankaRidgeback::PinocchioDynamics (pinocchio_dynamics.hpp:30-427) on the device.
    `create(initial_state)` runs the constructor's set_state (pinocchio_dynamics.cpp:84-115)."""
    STATE_DOF = abi.MPPI_FR_STATE
    CONTROL_DOF = abi.MPPI_FR_CONTROL

    def __init__(self, handle, descriptor):
        self._L = load()
        self._h = handle
        self._desc = descriptor

    @staticmethod
    def create(initial_state, model=None, device=0):
        from .trajectory import EngineError, FrankaRidgebackDynamics
        L = load()
        desc = FrankaRidgebackDynamics(model).descriptor()
        x = np.ascontiguousarray(initial_state, dtype=np.float64).reshape(-1)
        if x.size != abi.MPPI_FR_STATE:
            raise ValueError("initial state must have %d entries" % abi.MPPI_FR_STATE)
        h = C.c_void_p()
        st = L.mppi_dynamics_create(C.byref(desc), _p(x), int(device), C.byref(h))
        if st != abi.MPPI_OK:
            raise EngineError(st, L.mppi_last_error(None).decode())
        return PinocchioDynamicsObject(h, desc)

    def close(self):
        if getattr(self, "_h", None):
            self._L.mppi_dynamics_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != abi.MPPI_OK:
            from .trajectory import EngineError
            raise EngineError(st, self._L.mppi_last_error(None).decode())

    @property
    def handle(self):
        return self._h

    def copy(self):
        """mppi::Dynamics::copy (mppi.hpp:47): a new object at this one's state."""
        return PinocchioDynamicsObject.create(self.get_state())

    def set_state(self, state, time):
        x = np.ascontiguousarray(state, dtype=np.float64).reshape(-1)
        assert x.size == abi.MPPI_FR_STATE
        self._check(self._L.mppi_dynamics_set_state(self._h, _p(x), float(time)))

    def step(self, control, dt):
        """PinocchioDynamics::step (pinocchio_dynamics.cpp:226-260): the new state."""
        u = np.ascontiguousarray(control, dtype=np.float64).reshape(-1)
        assert u.size == abi.MPPI_FR_CONTROL
        out = np.zeros(abi.MPPI_FR_STATE)
        self._check(self._L.mppi_dynamics_step(self._h, _p(u), float(dt), _p(out)))
        return out

    def get_state(self):
        out = np.zeros(abi.MPPI_FR_STATE)
        self._check(self._L.mppi_dynamics_get_state(self._h, _p(out)))
        return out

    def get_end_effector_state_row(self):
        """The EndEffectorState as its MPPI_EE_N-double row."""
        out = np.zeros(abi.MPPI_EE_N)
        self._check(self._L.mppi_dynamics_end_effector(self._h, _p(out)))
        return out

    def get_end_effector_state(self):
        return EndEffectorState.from_row(self.get_end_effector_state_row())

    def query_row(self):
        """The members after the last call as MPPI_DYNAMICS_QUERY_N doubles."""
        o = np.zeros(abi.MPPI_DYNAMICS_QUERY_N)
        self._check(self._L.mppi_dynamics_query(self._h, _p(o)))
        return o

    def query(self):
        """dict of the members after the last call: joint position / velocity / acceleration /
        torque, tank energy, power, time, arm-mount frame position."""
        o = self.query_row()
        return {"joint_position": o[0:12], "joint_velocity": o[12:24], "joint_acceleration": o[24:36],
                "joint_torque": o[36:48], "tank_energy": o[48], "power": o[49], "time": o[50],
                "arm_mount_position": o[51:54]}

    def get_joint_position(self):
        return self.query()["joint_position"]

    def get_joint_velocity(self):
        return self.query()["joint_velocity"]

    def get_tank_energy(self):
        return self.query()["tank_energy"]

    def get_joint_power(self):
        return 0.0   # pinocchio_dynamics.hpp:211-214

    def get_external_power(self):
        return 0.0   # pinocchio_dynamics.hpp:220-223

    def get_control_dof(self):
        return abi.MPPI_FR_CONTROL

    def get_state_dof(self):
        return abi.MPPI_FR_STATE

    def forecast_rows(self, state, time, time_step, steps, wrench=None):
        """[steps x MPPI_DF_N] rows of DynamicsForecast::forecast (mppi_dynamics_forecast)."""
        x = np.ascontiguousarray(state, dtype=np.float64).reshape(-1)
        out = np.zeros((int(steps), abi.MPPI_DF_N))
        w = None if wrench is None else np.ascontiguousarray(wrench, dtype=np.float64).reshape(int(steps), 6)
        self._check(self._L.mppi_dynamics_forecast(self._h, _p(x), float(time), float(time_step), int(steps),
                                                   None if w is None else _p(w), _p(out)))
        return out


def evaluate_cost(cost, dynamics, state, control=None, wrench=None):
    """Cost::get_cost(state, control, dynamics, time) (mppi.hpp:127-132) on the device against a
    PinocchioDynamicsObject's cached kinematics; `wrench` = forecast(time) of the dynamics' forecast
    handle (None: no handle, trajectory_cost 0).  Returns (cost, seven AssistedManipulation terms)."""
    L = load()
    desc = cost.descriptor()
    x = np.ascontiguousarray(state, dtype=np.float64).reshape(-1)
    u = np.zeros(abi.MPPI_FR_CONTROL) if control is None else np.ascontiguousarray(control, dtype=np.float64)
    w = None if wrench is None else np.ascontiguousarray(wrench, dtype=np.float64).reshape(6)
    out = np.zeros(8)
    st = L.mppi_cost_evaluate(C.byref(desc), dynamics.handle, _p(x), _p(u), None if w is None else _p(w), _p(out))
    if st != abi.MPPI_OK:
        from .trajectory import EngineError
        raise EngineError(st, L.mppi_last_error(None).decode())
    return out[0], out[1:]


class DynamicsForecast:
    """FrankaRidgeback::DynamicsForecast (dynamics.hpp:122-387, dynamics.cpp:57-138).  The wrench
    forecast it owns in the reference is the trajectory's device forecast here (`source`: a
    Trajectory with mppi_forecast_attach done, the forecast the rollouts' trajectory cost reads, as
    the Actor shares one DynamicsForecast between both, actor.cpp:70-89).  forecast() is one
    device launch for the whole horison."""

    def __init__(self, time_step, horison, dynamics, source):
        import math
        self.time_step, self.horison = float(time_step), float(horison)
        self.steps = int(math.ceil(horison / time_step))
        if self.steps <= 0:
            raise ValueError("time horison is too small for time step")   # dynamics.cpp:70-74
        self.dynamics = dynamics
        self.source = source
        self.last_forecast = np.finfo(np.float64).tiny   # std::numeric_limits<double>::min()
        self.rows = np.zeros((self.steps, abi.MPPI_DF_N))

    def observe_wrench(self, wrench, time):
        self.source.observe_wrench(wrench, time)

    def observe_time(self, time):
        self.source.observe_time(time)

    def forecast(self, state, time):
        wrench = self.source.forecast_table(time, self.time_step, self.steps)
        self.rows = self.dynamics.forecast_rows(state, time, self.time_step, self.steps, wrench)
        self.last_forecast = float(time)

    def get_last_forecast_time(self):
        return self.last_forecast

    def parameterise(self, time):
        """dynamics.hpp:344-359, literally (the horison is compared with the absolute time)."""
        if time < self.last_forecast:
            return 0
        if time >= self.horison:
            return self.steps - 1
        return int((time - self.last_forecast) / self.time_step)

    def get_joint_position(self):
        return self.rows[:, abi.MPPI_DF_JOINT_POSITION:abi.MPPI_DF_JOINT_POSITION + 12].copy()

    def get_end_effector_state(self, time):
        k = self.parameterise(time)
        return EndEffectorState.from_row(self.rows[k, abi.MPPI_DF_END_EFFECTOR:abi.MPPI_DF_END_EFFECTOR + abi.MPPI_EE_N])

    def get_end_effector_wrench(self, time):
        return self.source.forecast(time)   # dynamics.hpp:275-278: the forecast itself, not the rows

    def get_end_effector_trajectory(self):
        return [EndEffectorState.from_row(r[abi.MPPI_DF_END_EFFECTOR:abi.MPPI_DF_END_EFFECTOR + abi.MPPI_EE_N])
                for r in self.rows]

    def get_wrench_trajectory(self):
        return self.rows[:, abi.MPPI_DF_WRENCH:abi.MPPI_DF_WRENCH + 6].copy()

    def get_joint_power_trajectory(self):
        return self.rows[:, abi.MPPI_DF_JOINT_POWER].copy()

    def get_external_power_trajectory(self):
        return self.rows[:, abi.MPPI_DF_EXTERNAL_POWER].copy()

    def get_energy_trajectory(self):
        return self.rows[:, abi.MPPI_DF_ENERGY].copy()

    def get_time_step(self):
        return self.time_step

    def get_horison(self):
        return self.horison
