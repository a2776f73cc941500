"""assistedmanipulation_amd — MI355X-native MPPI trajectory engine.

A drop-in for the reference's mppi::Trajectory hot path (LuigiVan01/AssistedManipulation,
src/controller/mppi.{hpp,cpp}) with the FrankaRidgeback Pinocchio dynamics and the
AssistedManipulation cost evaluated by hand-written HIP kernels for gfx950.  The native
library (lib/libmppi_amd.so, C-ABI in include/mppi_amd.h) is loaded at import; there is no
CPU fallback.
"""
from . import abi
from ._lib import load as _load

_load()   # fail loudly at import if the engine library is missing

from .config import (Configuration, Smoothing, average_forecast_configuration, constant_forecast,  # noqa: E402
                     frankaridgeback_configuration, huddled_state, kalman_forecast_configuration,
                     locf_forecast_configuration, point_mass_configuration)
from .trajectory import (AssistedManipulation, Cost, Dynamics, EngineError, TrackPoint,  # noqa: E402
                         FrankaRidgebackDynamics, PointMassDynamics, QuadraticCost, Trajectory,
                         comm_unique_id, shard_range)

from .csvlog import MPPILogger  # noqa: E402
from .dynamics import DynamicsForecast, EndEffectorState, PinocchioDynamicsObject, evaluate_cost  # noqa: E402

__all__ = [
    "MPPILogger", "DynamicsForecast", "EndEffectorState", "PinocchioDynamicsObject", "evaluate_cost",
    "abi", "Configuration", "Smoothing", "constant_forecast", "frankaridgeback_configuration",
    "huddled_state", "point_mass_configuration", "locf_forecast_configuration", "average_forecast_configuration",
    "kalman_forecast_configuration", "AssistedManipulation", "TrackPoint", "Cost", "Dynamics",
    "EngineError", "FrankaRidgebackDynamics", "PointMassDynamics", "QuadraticCost", "Trajectory",
    "comm_unique_id", "shard_range",
]
