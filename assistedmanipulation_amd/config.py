"""Host-side mirror of mppi::Configuration (src/controller/mppi.hpp:181-249) and builders for
the dynamics / cost descriptors that replace the reference's plugin objects.

`Configuration` keeps the reference's field names, meaning and defaults; `to_c()` produces the
POD `mppi_config` the C-ABI takes (plus the numpy arrays it points into, which the caller must
keep alive for the duration of the call).
"""
import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi


@dataclass
class Smoothing:
    """mppi::Configuration::Smoothing (mppi.hpp:223-233)."""
    window: int = 10
    order: int = 1


@dataclass
class Configuration:
    """mppi::Configuration, field for field."""
    initial_state: np.ndarray
    rollouts: int
    keep_best_rollouts: int
    time_step: float
    horison: float
    gradient_step: float
    cost_scale: float
    cost_discount_factor: float
    covariance: np.ndarray
    control_bound: bool
    control_min: np.ndarray
    control_max: np.ndarray
    control_default: Optional[np.ndarray] = None
    smoothing: Optional[Smoothing] = None
    threads: int = 1

    @property
    def steps(self):
        """H = ceil(horison / time_step) (mppi.cpp:85)."""
        return int(math.ceil(self.horison / self.time_step))

    def to_c(self):
        """Return (mppi_config, keepalive) — keepalive holds the arrays the struct points to."""
        keep = []

        def arr(x):
            a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(C.c_double))

        cov = np.asarray(self.covariance, dtype=np.float64)
        n = cov.shape[0]
        c = abi.mppi_config()
        c.initial_state = arr(self.initial_state)
        c.state_dof = int(np.asarray(self.initial_state).size)
        c.control_dof = int(n)
        c.rollouts = int(self.rollouts)
        c.keep_best_rollouts = int(self.keep_best_rollouts)
        c.time_step = float(self.time_step)
        c.horison = float(self.horison)
        c.gradient_step = float(self.gradient_step)
        c.cost_scale = float(self.cost_scale)
        c.cost_discount_factor = float(self.cost_discount_factor)
        c.covariance = arr(cov.T)   # column-major (Eigen)
        c.control_bound = int(bool(self.control_bound))
        c.control_min = arr(self.control_min)
        c.control_max = arr(self.control_max)
        c.has_control_default = int(self.control_default is not None)
        c.control_default = arr(self.control_default) if self.control_default is not None else None
        c.has_smoothing = int(self.smoothing is not None)
        c.smoothing_window = int(self.smoothing.window) if self.smoothing else 0
        c.smoothing_order = int(self.smoothing.order) if self.smoothing else 0
        c.threads = int(self.threads)
        return c, keep


FR_VARIANCE = np.array([0.1, 0.1, 0.2] + [7.5] * 7 + [0.0, 0.0])
FR_CONTROL_MIN = np.array([-0.5, -0.5, -1.0] + [-100.0] * 7 + [-0.05, -0.05])
FR_CONTROL_MAX = -FR_CONTROL_MIN


def huddled_state():
    """make_state(Preset::HUDDLED) (frankaridgeback/state.cpp:15-18)."""
    x = np.zeros(abi.MPPI_FR_STATE)
    x[:12] = [0.2, 0.2, math.pi / 4, 0.0, math.pi / 5, 0.0, -math.pi / 2, 0.0, 2, math.pi / 4, 0.025, 0.025]
    x[30] = 100.0
    return x


def frankaridgeback_configuration(rollouts=50, horison=0.3, keep_best_rollouts=20, smoothing=None,
                                  threads=1, time_step=0.01):
    """BaseTest::DEFAULT_CONFIGURATION's mppi block (test/case/base.hpp:69-101).  `smoothing`
    defaults to None here (off for configs 1-4); pass Smoothing() for config 5."""
    return Configuration(
        initial_state=huddled_state(), rollouts=rollouts, keep_best_rollouts=keep_best_rollouts,
        time_step=time_step, horison=horison, gradient_step=2.0, cost_scale=10.0,
        cost_discount_factor=1.0, covariance=np.diag(FR_VARIANCE), control_bound=True,
        control_min=FR_CONTROL_MIN.copy(), control_max=FR_CONTROL_MAX.copy(),
        control_default=np.zeros(abi.MPPI_FR_CONTROL), smoothing=smoothing, threads=threads)


def point_mass_configuration(rollouts=1024, horison=0.32, keep_best_rollouts=20, time_step=0.01):
    """Config 2: point mass, C = 3, Sigma = 0.5^2 I, x0 = 0."""
    return Configuration(
        initial_state=np.zeros(6), rollouts=rollouts, keep_best_rollouts=keep_best_rollouts,
        time_step=time_step, horison=horison, gradient_step=2.0, cost_scale=10.0,
        cost_discount_factor=1.0, covariance=np.eye(3) * 0.25, control_bound=True,
        control_min=-np.ones(3) * 5.0, control_max=np.ones(3) * 5.0,
        control_default=np.zeros(3), smoothing=None, threads=1)


def point_mass_dynamics(mass=1.0):
    d = abi.mppi_dynamics_desc()
    d.kind = abi.MPPI_DYNAMICS_POINT_MASS
    d.point_mass.mass = mass
    return d


def quadratic_cost(target=(1.0, 1.0, 1.0), q=(1.0, 1.0, 1.0), r=(0.01, 0.01, 0.01)):
    c = abi.mppi_cost_desc()
    c.kind = abi.MPPI_COST_QUADRATIC
    for i in range(3):
        c.quadratic.target[i] = target[i]
        c.quadratic.q[i] = q[i]
        c.quadratic.r[i] = r[i]
    return c


def frankaridgeback_dynamics(model_desc):
    """Wrap a mppi_frankaridgeback_desc (e.g. from mppi_default_frankaridgeback)."""
    d = abi.mppi_dynamics_desc()
    d.kind = abi.MPPI_DYNAMICS_FRANKARIDGEBACK
    d.frankaridgeback = model_desc
    return d


def assisted_manipulation_cost(am_desc):
    c = abi.mppi_cost_desc()
    c.kind = abi.MPPI_COST_ASSISTED_MANIPULATION
    c.assisted_manipulation = am_desc
    return c


def constant_forecast(H, force=(20.0, 0.0, 0.0)):
    """Per-update forecast table: constant wrench F = (20, 0, 0, 0, 0, 0) N."""
    t = np.zeros((H, 6))
    t[:, :3] = force
    return t


def locf_forecast_configuration(observation=(0.0,) * 6, horison=0.0):
    """LOCFForecast::Configuration (forecast.hpp:66-76)."""
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_LOCF
    c.locf_observation[:] = list(observation)
    c.locf_horison = horison
    return c


def average_forecast_configuration(window, states=6):
    """AverageForecast::Configuration (forecast.hpp:151-161)."""
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_AVERAGE
    c.average_states = states
    c.average_window = window
    return c


def kalman_forecast_configuration(time_step, horison, order, initial_state=(0.0,) * 6, observed_states=6):
    """KalmanForecast::Configuration (forecast.hpp:227-249)."""
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_KALMAN
    c.kalman_observed_states = observed_states
    c.kalman_time_step = time_step
    c.kalman_horison = horison
    c.kalman_order = order
    c.kalman_initial_state[:] = list(initial_state)
    return c
