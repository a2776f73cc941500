"""ctypes wrapper of oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline.  The product (assistedmanipulation_amd) never does.
The oracle restates the reference's fp64 CPU path (see oracle/mppi_oracle.cpp's header).
"""
import ctypes as C
import os
import subprocess

import numpy as np

from assistedmanipulation_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
_lib = None
ALLREDUCE_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int64)


def build(native=False):
    """Compile the oracle (make).  native=True builds with -march=native into build-native/."""
    if native:
        out = os.path.join(HERE, "build-native")
        os.makedirs(out, exist_ok=True)
        subprocess.check_call(["make", "-s", "-C", HERE, "ARCH=native", "OUT=build-native"])
        return os.path.join(out, "liboracle.so")
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib(path=None):
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        build()
    L = C.CDLL(p)
    vp, dp, i64 = C.c_void_p, C.POINTER(C.c_double), C.c_int64
    L.oracle_create.restype = vp
    L.oracle_create.argtypes = [C.POINTER(abi.mppi_config), C.POINTER(abi.mppi_dynamics_desc),
                                C.POINTER(abi.mppi_cost_desc), C.c_int, C.c_int, C.c_int]
    L.oracle_last_error.restype = C.c_char_p
    L.oracle_last_error.argtypes = [vp]
    L.oracle_destroy.argtypes = [vp]
    L.oracle_set_noise_source.argtypes = [vp, C.c_int, C.c_uint64]
    L.oracle_inject_noise.argtypes = [vp, dp, i64]
    L.oracle_noise_draws.restype = i64
    L.oracle_noise_draws.argtypes = [vp, C.c_double]
    L.oracle_set_forecast.argtypes = [vp, dp]
    L.oracle_update.argtypes = [vp, dp, C.c_double]
    L.oracle_get.argtypes = [vp, C.c_double, dp]
    L.oracle_dims.argtypes = [vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
    for n in ("oracle_costs", "oracle_weights", "oracle_gradient", "oracle_optimal_control",
              "oracle_noise", "oracle_optimal_terms", "oracle_set_costs"):
        getattr(L, n).argtypes = [vp, dp]
    L.oracle_optimal_cost.restype = C.c_double
    L.oracle_optimal_cost.argtypes = [vp]
    L.oracle_update_duration.restype = C.c_double
    L.oracle_update_duration.argtypes = [vp]
    L.oracle_set_threads.argtypes = [vp, C.c_uint]
    L.oracle_set_shard.argtypes = [vp, i64, i64, ALLREDUCE_FN]
    L.oracle_smoothing_windows.argtypes = [vp, dp, dp, C.POINTER(C.c_int64)]
    L.oracle_kinematics.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc), dp, dp, dp, C.c_int, dp]
    L.oracle_rollout.restype = C.c_double
    L.oracle_rollout.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc),
                                 C.POINTER(abi.mppi_assisted_manipulation_desc), dp, dp, i64,
                                 C.c_double, C.c_double, dp, C.c_int, C.c_int, dp, dp]
    L.oracle_count_flops_split.restype = C.c_double
    L.oracle_count_flops_split.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc),
                                           C.POINTER(abi.mppi_assisted_manipulation_desc), dp, C.c_int64, dp]
    L.oracle_count_flops_phases.restype = C.c_double
    L.oracle_count_flops_phases.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc),
                                            C.POINTER(abi.mppi_assisted_manipulation_desc), dp, C.c_int64, dp]
    L.oracle_count_flops.restype = C.c_double
    L.oracle_count_flops.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc),
                                     C.POINTER(abi.mppi_assisted_manipulation_desc), dp, i64]
    L.oracle_sg_weights.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp]
    L.oracle_default_frankaridgeback.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc)]
    L.oracle_default_assisted_manipulation.argtypes = [C.POINTER(abi.mppi_assisted_manipulation_desc)]
    L.oracle_dyn_create.restype = vp
    L.oracle_dyn_create.argtypes = [C.POINTER(abi.mppi_frankaridgeback_desc), dp]
    L.oracle_dyn_destroy.argtypes = [vp]
    L.oracle_dyn_set_state.argtypes = [vp, dp, C.c_double]
    L.oracle_dyn_step.argtypes = [vp, dp, C.c_double, dp]
    for n in ("oracle_dyn_get_state", "oracle_dyn_end_effector", "oracle_dyn_query"):
        getattr(L, n).argtypes = [vp, dp]
    L.oracle_dyn_forecast.argtypes = [vp, dp, C.c_double, C.c_double, C.c_int64, dp, dp]
    L.oracle_cost_evaluate.argtypes = [C.POINTER(abi.mppi_cost_desc), vp, dp, dp, dp]
    L.oracle_forecast_create.restype = vp
    L.oracle_forecast_create.argtypes = [C.POINTER(abi.mppi_forecast_config), C.c_char_p, C.c_int]
    L.oracle_forecast_destroy.argtypes = [vp]
    L.oracle_forecast_observe.argtypes = [vp, dp, C.c_double]
    L.oracle_forecast_observe_time.argtypes = [vp, C.c_double]
    L.oracle_forecast_get.argtypes = [vp, C.c_double, dp]
    if path is None:
        _lib = L
    return L


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def default_model():
    d = abi.mppi_frankaridgeback_desc()
    lib().oracle_default_frankaridgeback(C.byref(d))
    return d


def default_cost():
    a = abi.mppi_assisted_manipulation_desc()
    lib().oracle_default_assisted_manipulation(C.byref(a))
    return a


def kinematics(model, q, v, tau, mode=0):
    """calculate() probe: dict of a, ee, arm_mount, J (6x12), v_ee (6), nle (12); mode 0 also the
    EE rotation (3x3) and WORLD spatial acceleration a_ee (6)."""
    out = np.zeros(12 + 3 + 3 + 72 + 6 + 12 + 15)
    q, v, tau = (np.ascontiguousarray(x, dtype=np.float64) for x in (q, v, tau))
    lib().oracle_kinematics(C.byref(model), _p(q), _p(v), _p(tau), mode, _p(out))
    return dict(a=out[:12], ee=out[12:15], arm_mount=out[15:18], J=out[18:90].reshape(6, 12),
                v_ee=out[90:96], nle=out[96:108], R_ee=out[108:117].reshape(3, 3), a_ee=out[117:123])


def rollout(model, cost, x0, u_HxC, dt, t0=0.0, forecast=None, scalar=0, mode=0):
    H = u_HxC.shape[0]
    u = np.ascontiguousarray(u_HxC, dtype=np.float64)
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    sc = np.zeros(H)
    xf = np.zeros(abi.MPPI_FR_STATE)
    f = None if forecast is None else np.ascontiguousarray(forecast, dtype=np.float64)
    total = lib().oracle_rollout(C.byref(model), C.byref(cost), _p(x0), _p(u), H, dt, t0,
                                 None if f is None else _p(f), scalar, mode, _p(sc), _p(xf))
    return total, sc, xf


def count_flops_split(model, cost, x0, steps=64):
    """(total, cost part) algorithmic FLOPs per rollout-step; total - cost is the rollout kernel's."""
    part = C.c_double(0.0)
    tot = lib().oracle_count_flops_split(C.byref(model), C.byref(cost), _p(x0), steps, C.byref(part))
    return tot, part.value


FLOP_PHASES = ("fk", "world_inertia", "solve", "kinematics", "integration", "objective")


def count_flops_phases(model, cost, x0, steps=64):
    """(total, {phase: FLOPs}) algorithmic FLOPs per rollout-step by phase (FLOP_PHASES)."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    out = np.zeros(6)
    tot = lib().oracle_count_flops_phases(C.byref(model), C.byref(cost), _p(x0), steps, _p(out))
    return tot, dict(zip(FLOP_PHASES, out.tolist()))


def count_flops(model, cost, x0, steps=64):
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    return lib().oracle_count_flops(C.byref(model), C.byref(cost), _p(x0), steps)


def sg_weights(m, t, n, s):
    out = np.zeros(2 * m + 1)
    lib().oracle_sg_weights(m, t, n, s, _p(out))
    return out


class OracleTrajectory:
    """mppi::Trajectory restated on the CPU (fp64).  scalar=1 runs dynamics/cost in float,
    mode=1 uses the minimal-arithmetic (zero-bias, world-frame ABA) dynamics."""

    def __init__(self, config_c, dynamics_desc, cost_desc, scalar=0, mode=0, compat_uint8=0,
                 lib_path=None):
        self._L = lib(lib_path) if lib_path else lib()
        self._h = self._L.oracle_create(C.byref(config_c), C.byref(dynamics_desc),
                                        C.byref(cost_desc), scalar, mode, compat_uint8)
        if not self._h:
            raise ValueError(self._L.oracle_last_error(None).decode())
        R, H, Cc, X = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        self._L.oracle_dims(self._h, C.byref(R), C.byref(H), C.byref(Cc), C.byref(X))
        self.R, self.H, self.C, self.X = R.value, H.value, Cc.value, X.value

    def close(self):
        if self._h:
            self._L.oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_noise_source(self, injected, seed=0):
        self._L.oracle_set_noise_source(self._h, int(injected), seed)

    def inject_noise(self, eps):
        eps = np.ascontiguousarray(eps, dtype=np.float64).reshape(-1)
        self._L.oracle_inject_noise(self._h, _p(eps), eps.size // self.C)

    def noise_draws(self, time):
        return self._L.oracle_noise_draws(self._h, time)

    def set_forecast(self, table):
        if table is None:
            self._L.oracle_set_forecast(self._h, None)
        else:
            t = np.ascontiguousarray(table, dtype=np.float64)
            self._forecast_keep = t
            self._L.oracle_set_forecast(self._h, _p(t))

    def set_shard(self, begin, end, allreduce):
        """Sharded mode: roll out [begin, end) only; `allreduce(ptr, n)` sums n doubles in place
        across ranks (called for the cost vector and the partial gradient)."""
        self._allreduce_cb = ALLREDUCE_FN(allreduce)
        self._L.oracle_set_shard(self._h, begin, end, self._allreduce_cb)

    def set_threads(self, n):
        self._L.oracle_set_threads(self._h, n)

    def update(self, state, time):
        s = np.ascontiguousarray(state, dtype=np.float64)
        st = self._L.oracle_update(self._h, _p(s), time)
        if st != 0:
            raise RuntimeError("%s: %s" % (abi.STATUS_NAMES.get(st, st),
                                           self._L.oracle_last_error(self._h).decode()))

    def get(self, time):
        out = np.zeros(self.C)
        st = self._L.oracle_get(self._h, time, _p(out))
        if st != 0:
            raise RuntimeError(abi.STATUS_NAMES.get(st, st))
        return out

    def _vec(self, name, n):
        out = np.zeros(n)
        getattr(self._L, name)(self._h, _p(out))
        return out

    def costs(self):
        return self._vec("oracle_costs", self.R)

    def set_costs(self, costs):
        """Test hook: the previous costs the next sample() sorts (oracle_set_costs)."""
        c = np.ascontiguousarray(costs, dtype=np.float64)
        assert c.size == self.R
        self._L.oracle_set_costs(self._h, _p(c))

    def weights(self):
        return self._vec("oracle_weights", self.R)

    def gradient(self):
        return self._vec("oracle_gradient", self.C * self.H).reshape(self.H, self.C)

    def optimal_control(self):
        return self._vec("oracle_optimal_control", self.C * self.H).reshape(self.H, self.C)

    def noise(self):
        return self._vec("oracle_noise", self.R * self.C * self.H).reshape(self.R, self.H, self.C)

    def optimal_terms(self):
        return self._vec("oracle_optimal_terms", 7)

    def smoothing_windows(self, window):
        W = self.H + 2 * window + 1
        uu, tt = np.zeros((self.C, W)), np.zeros((self.C, W))
        st = np.zeros(self.C, dtype=np.int64)
        self._L.oracle_smoothing_windows(self._h, _p(uu), _p(tt), st.ctypes.data_as(C.POINTER(C.c_int64)))
        return uu, tt, st

    def optimal_cost(self):
        return self._L.oracle_optimal_cost(self._h)

    def update_duration(self):
        return self._L.oracle_update_duration(self._h)


class OracleDynamics:
    """FrankaRidgeback::PinocchioDynamics as an object (pinocchio_dynamics.cpp:84-260), restated:
    the checker of the engine's mppi_dynamics_* (tests/test_gpu_dynamics.py)."""

    def __init__(self, initial_state, model=None):
        self._L = lib()
        self._model = model if model is not None else default_model()
        x = np.ascontiguousarray(initial_state, dtype=np.float64)
        self._h = self._L.oracle_dyn_create(C.byref(self._model), _p(x))

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.oracle_dyn_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def set_state(self, x, time):
        x = np.ascontiguousarray(x, dtype=np.float64)
        self._L.oracle_dyn_set_state(self._h, _p(x), float(time))

    def step(self, u, dt):
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(abi.MPPI_FR_STATE)
        self._L.oracle_dyn_step(self._h, _p(u), float(dt), _p(out))
        return out

    def get_state(self):
        out = np.zeros(abi.MPPI_FR_STATE)
        self._L.oracle_dyn_get_state(self._h, _p(out))
        return out

    def end_effector(self):
        out = np.zeros(abi.MPPI_EE_N)
        self._L.oracle_dyn_end_effector(self._h, _p(out))
        return out

    def query(self):
        out = np.zeros(abi.MPPI_DYNAMICS_QUERY_N)
        self._L.oracle_dyn_query(self._h, _p(out))
        return out

    def forecast_rows(self, x, time, time_step, steps, wrench=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros((int(steps), abi.MPPI_DF_N))
        w = None if wrench is None else np.ascontiguousarray(wrench, dtype=np.float64)
        self._L.oracle_dyn_forecast(self._h, _p(x), float(time), float(time_step), int(steps),
                                    None if w is None else _p(w), _p(out))
        return out

    def evaluate_cost(self, cost_desc, x, wrench=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        w = None if wrench is None else np.ascontiguousarray(wrench, dtype=np.float64)
        out = np.zeros(8)
        self._L.oracle_cost_evaluate(C.byref(cost_desc), self._h, _p(x), None if w is None else _p(w), _p(out))
        return out[0], out[1:]


class OracleForecast:
    """controller/forecast.{hpp,cpp} + kalman.cpp restated (oracle/forecast_oracle.cpp)."""

    def __init__(self, config):
        self._L = lib()
        err = C.create_string_buffer(256)
        self._h = self._L.oracle_forecast_create(C.byref(config), err, 256)
        self.error = err.value.decode()
        if not self._h:
            raise ValueError(self.error)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.oracle_forecast_destroy(self._h)
            self._h = None

    def observe(self, wrench, time):
        w = np.ascontiguousarray(wrench, dtype=np.float64)
        self._L.oracle_forecast_observe(self._h, _p(w), float(time))

    def observe_time(self, time):
        self._L.oracle_forecast_observe_time(self._h, float(time))

    def get(self, time):
        out = np.zeros(6)
        self._L.oracle_forecast_get(self._h, float(time), _p(out))
        return out

    def table(self, t0, dt, H):
        """[H x 6]: forecast(t0 + k dt), what the rollout's cost queries at step k."""
        return np.array([self.get(t0 + k * dt) for k in range(H)])
