"""mppi::Trajectory and its plugin surface on the MI355X engine.

Mirrors src/controller/mppi.hpp of the reference: `Trajectory.create(configuration, dynamics,
cost)` returns None on a validation failure (the reference returns nullptr and prints to stderr,
mppi.cpp:17-69); `update(state, time)` runs one MPPI iteration on the device; `get(control,
time)` / `__call__(time)` interpolate the published optimal control; the accessors return the
quantities logger::MPPI records (logging/mppi.cpp:84-136).

The dynamics and cost are *descriptors* (POD parameter blocks) rather than virtual objects: the
kernels evaluate them on the device.  FrankaRidgebackDynamics / AssistedManipulation replace
FrankaRidgeback::PinocchioDynamics / FrankaRidgeback::AssistedManipulation;
PointMassDynamics / QuadraticCost are the bring-up plugins of SURVEY §8a a16.
"""
import ctypes as C
import sys

import numpy as np

from . import abi
from ._lib import load
from .config import Configuration


class EngineError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("%s: %s" % (abi.STATUS_NAMES.get(status, status), message))
        self.status = status


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


# ---- plugin descriptors -------------------------------------------------------------------
class Dynamics:
    """mppi::Dynamics (mppi.hpp:30-85) as a device descriptor."""
    control_dof = None
    state_dof = None

    def descriptor(self):
        raise NotImplementedError

    def get_control_dof(self):
        return self.control_dof

    def get_state_dof(self):
        return self.state_dof


class Cost:
    """mppi::Cost (mppi.hpp:93-145) as a device descriptor."""
    control_dof = None
    state_dof = None

    def descriptor(self):
        raise NotImplementedError

    def get_control_dof(self):
        return self.control_dof

    def get_state_dof(self):
        return self.state_dof


class FrankaRidgebackDynamics(Dynamics):
    """FrankaRidgeback::PinocchioDynamics (pinocchio_dynamics.{hpp,cpp}).  `model` is a
    mppi_frankaridgeback_desc; by default the body table generated from robot.urdf."""
    control_dof = abi.MPPI_FR_CONTROL
    state_dof = abi.MPPI_FR_STATE

    def __init__(self, model=None):
        if model is None:
            model = abi.mppi_frankaridgeback_desc()
            load().mppi_default_frankaridgeback(C.byref(model))
        self.model = model

    def descriptor(self):
        d = abi.mppi_dynamics_desc()
        d.kind = abi.MPPI_DYNAMICS_FRANKARIDGEBACK
        d.frankaridgeback = self.model
        return d


class PointMassDynamics(Dynamics):
    control_dof = 3
    state_dof = 6

    def __init__(self, mass=1.0):
        self.mass = mass

    def descriptor(self):
        d = abi.mppi_dynamics_desc()
        d.kind = abi.MPPI_DYNAMICS_POINT_MASS
        d.point_mass.mass = self.mass
        return d


class AssistedManipulation(Cost):
    """FrankaRidgeback::AssistedManipulation (objective/assisted_manipulation.{hpp,cpp}).
    `configuration` is a mppi_assisted_manipulation_desc; by default DEFAULT_CONFIGURATION."""
    control_dof = abi.MPPI_FR_CONTROL
    state_dof = abi.MPPI_FR_STATE

    def __init__(self, configuration=None):
        if configuration is None:
            configuration = abi.mppi_assisted_manipulation_desc()
            load().mppi_default_assisted_manipulation(C.byref(configuration))
        self.configuration = configuration

    def descriptor(self):
        c = abi.mppi_cost_desc()
        c.kind = abi.MPPI_COST_ASSISTED_MANIPULATION
        c.assisted_manipulation = self.configuration
        return c


class TrackPoint(Cost):
    """FrankaRidgeback::TrackPoint (objective/track_point.{hpp,cpp}).
    `configuration` is a mppi_track_point_desc; by default DEFAULT_CONFIGURATION; `point`
    overrides the tracked point."""
    control_dof = abi.MPPI_FR_CONTROL
    state_dof = abi.MPPI_FR_STATE

    def __init__(self, configuration=None, point=None):
        if configuration is None:
            configuration = abi.mppi_track_point_desc()
            load().mppi_default_track_point(C.byref(configuration))
        if point is not None:
            for i in range(3):
                configuration.point[i] = float(point[i])
        self.configuration = configuration

    def descriptor(self):
        c = abi.mppi_cost_desc()
        c.kind = abi.MPPI_COST_TRACK_POINT
        c.track_point = self.configuration
        return c


class QuadraticCost(Cost):
    control_dof = 3
    state_dof = 6

    def __init__(self, target=(1.0, 1.0, 1.0), q=(1.0, 1.0, 1.0), r=(0.01, 0.01, 0.01)):
        self.target, self.q, self.r = target, q, r

    def descriptor(self):
        c = abi.mppi_cost_desc()
        c.kind = abi.MPPI_COST_QUADRATIC
        for i in range(3):
            c.quadratic.target[i] = self.target[i]
            c.quadratic.q[i] = self.q[i]
            c.quadratic.r[i] = self.r[i]
        return c


def shard_range(rollout_count, world, rank):
    b, e = C.c_int64(), C.c_int64()
    st = load().mppi_shard_range(rollout_count, world, rank, C.byref(b), C.byref(e))
    if st != abi.MPPI_OK:
        raise EngineError(st, "invalid shard (%d, %d, %d)" % (rollout_count, world, rank))
    return b.value, e.value


def comm_unique_id():
    buf = C.create_string_buffer(128)
    st = load().mppi_comm_unique_id(buf)
    if st != abi.MPPI_OK:
        raise EngineError(st, "ncclGetUniqueId failed")
    return buf.raw


class CUpdateEntry(tuple):
    """(fn, handle, state pointer) of Trajectory.c_update_entry, holding the Trajectory alive."""

    def __new__(cls, items, trajectory):
        t = super().__new__(cls, items)
        t.trajectory = trajectory
        return t


class Trajectory:
    """mppi::Trajectory (mppi.hpp:267-658) on one MI355X device."""

    def __init__(self, handle, configuration, dynamics, cost):
        self._L = load()
        self._h = handle
        self.configuration = configuration
        self.dynamics = dynamics
        self.cost = cost
        R, H, Cc, X = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        self._check(self._L.mppi_dims(self._h, C.byref(R), C.byref(H), C.byref(Cc), C.byref(X)))
        self.R, self.H, self.C, self.X = R.value, H.value, Cc.value, X.value
        self._rolled_out_state = np.asarray(configuration.initial_state, dtype=np.float64).copy()
        self._rolled_out_state[:] = 0.0   # m_rollout_state.setZero() (mppi.cpp:121)
        self._state_buf = np.zeros(self.X, dtype=np.float64)
        self._state_ptr = _p(self._state_buf)

    @staticmethod
    def create(configuration: Configuration, dynamics: Dynamics, cost: Cost, device=0):
        """Trajectory::create — None (and a message on stderr) on invalid input."""
        L = load()
        cfg, keep = configuration.to_c()
        dd, cd = dynamics.descriptor(), cost.descriptor()
        h = C.c_void_p()
        st = L.mppi_create(C.byref(cfg), C.byref(dd), C.byref(cd), int(device), C.byref(h))
        del keep
        if st != abi.MPPI_OK:
            print(L.mppi_last_error(None).decode(), file=sys.stderr)
            return None
        return Trajectory(h, configuration, dynamics, cost)

    # -- lifecycle --------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.mppi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != abi.MPPI_OK:
            raise EngineError(st, self._L.mppi_last_error(self._h).decode())

    # -- multi-GPU ---------------------------------------------------------------------------
    def comm_init(self, world, rank, unique_id):
        self._check(self._L.mppi_comm_init(self._h, world, rank, unique_id))

    def comm_info(self):
        """The engine communicator as RCCL reports it: {"nranks", "rank"} (0 / -1 without one), and
        the handle's HIP device and PCI bus id (mppi_comm_info)."""
        n, r, d = C.c_int(), C.c_int(), C.c_int()
        bus = C.create_string_buffer(64)
        self._check(self._L.mppi_comm_info(self._h, C.byref(n), C.byref(r), C.byref(d), bus, 64))
        return {"nranks": n.value, "rank": r.value, "device": d.value, "pci_bus_id": bus.value.decode()}

    def set_shard(self, world, rank):
        self._check(self._L.mppi_set_shard(self._h, world, rank))

    # -- parity hooks ------------------------------------------------------------------------
    def set_noise_source(self, source, seed=0x5EED):
        self._check(self._L.mppi_set_noise_source(self._h, int(source), int(seed)))

    def inject_noise(self, eps):
        e = np.ascontiguousarray(eps, dtype=np.float64).reshape(-1)
        self._check(self._L.mppi_inject_noise(self._h, _p(e), e.size // self.C))

    def noise_draws(self, time):
        n = C.c_int64()
        self._check(self._L.mppi_noise_draws(self._h, float(time), C.byref(n)))
        return n.value

    def set_index_semantics(self, semantics):
        self._check(self._L.mppi_set_index_semantics(self._h, int(semantics)))

    def set_forecast(self, wrench_Hx6):
        if wrench_Hx6 is None:
            self._check(self._L.mppi_set_forecast(self._h, None))
            return
        t = np.ascontiguousarray(wrench_Hx6, dtype=np.float64)
        assert t.shape == (self.H, 6), t.shape
        self._check(self._L.mppi_set_forecast(self._h, _p(t)))

    # -- device wrench forecast -------------------------------------------
    def attach_forecast(self, configuration):
        """Forecast::create bound to the engine (forecast.cpp:6-39): every update then samples
        forecast(t0 + k dt) on the device.  None detaches (back to set_forecast tables)."""
        self._check(self._L.mppi_forecast_attach(self._h, None if configuration is None else C.byref(configuration)))

    def observe_wrench(self, wrench, time):
        """DynamicsForecast::observe_wrench (dynamics.hpp:221-224)."""
        w = np.ascontiguousarray(wrench, dtype=np.float64)
        assert w.size == 6
        self._check(self._L.mppi_forecast_observe(self._h, _p(w), float(time)))

    def observe_time(self, time):
        """DynamicsForecast::observe_time (dynamics.hpp:231-234)."""
        self._check(self._L.mppi_forecast_observe_time(self._h, float(time)))

    def forecast(self, time):
        """Forecast::forecast(time): the wrench the rollout's cost sees at `time`."""
        out = np.zeros(6)
        self._check(self._L.mppi_forecast_get(self._h, float(time), _p(out)))
        return out

    def forecast_table(self, t0, dt, steps):
        """[steps x 6]: forecast(t0 + k dt) of the attached device forecast (mppi_forecast_table)."""
        out = np.zeros((int(steps), 6))
        self._check(self._L.mppi_forecast_table(self._h, float(t0), float(dt), int(steps), _p(out)))
        return out

    def step_constants(self):
        """Parity hook: [H x 8] per-step trajectory-cost constants of the last update."""
        out = np.zeros((self.H, 8))
        self._check(self._L.mppi_step_constants(self._h, _p(out)))
        return out

    # -- the hot path ------------------------------------------------------------------------
    def update(self, state, time):
        """Trajectory::update (mppi.cpp:154-187)."""
        buf = self._state_buf   # one contiguous buffer and its pointer, built once: the update
        if type(state) is np.ndarray and state.shape == buf.shape:   # path is latency-bound: the usual
            buf[...] = state                                         # case in one copy (~0.7 us, not ~2.6)
        else:
            if np.size(state) != self.X:
                raise ValueError("state must have %d entries, got %d" % (self.X, np.size(state)))
            np.copyto(buf, np.reshape(state, -1))
        st = self._L.mppi_update(self._h, self._state_ptr, float(time))
        if st != abi.MPPI_OK:
            self._check(st)
        self._rolled_out_state = buf   # copied when queried (get_rolled_out_state)

    def c_update_entry(self, state):
        """The C-ABI update entry for a caller that drives its own loop, as a C++ caller of
        include/mppi_amd.hpp does: returns (fn, handle, state pointer), with `state` copied into
        the handle's state buffer once; fn(handle, pointer, time) is mppi_update (mppi.cpp:154-187)
        and returns an mppi_status (abi.MPPI_OK = 0).  Change the state by writing the buffer
        (self.state_buffer) in place.  The update count and time live in the engine
        (get_update_count / get_update_last read them), so updates made through it count.
        Lifetime: the handle and the pointer are this Trajectory's; the returned entry holds a
        reference to it (entry.trajectory), so keep the entry - or the Trajectory - alive while
        calling fn (after close() or garbage collection the handle is freed)."""
        buf = self._state_buf
        if np.size(state) != self.X:
            raise ValueError("state must have %d entries, got %d" % (self.X, np.size(state)))
        np.copyto(buf, np.reshape(np.asarray(state, dtype=np.float64), -1))
        self._rolled_out_state = buf
        return CUpdateEntry((self._L.mppi_update, self._h, self._state_ptr), self)

    @property
    def state_buffer(self):
        """The state buffer c_update_entry's pointer points at."""
        return self._state_buf

    def set_graph(self, enable):
        """The hipGraph path of update() (mppi_set_graph): the steady-state update as one graph launch."""
        self._check(self._L.mppi_set_graph(self._h, int(bool(enable))))

    def graph_updates(self):
        """How many updates ran as the captured graph (mppi_graph_updates)."""
        n = C.c_int64()
        self._check(self._L.mppi_graph_updates(self._h, C.byref(n)))
        return n.value

    def synchronize(self):
        """Wait for all device work of this handle (including the overlapped filter())."""
        self._check(self._L.mppi_synchronize(self._h))

    def update_phase1(self, state, time):
        s = np.ascontiguousarray(state, dtype=np.float64).reshape(-1)
        if s.size != self.X:
            raise ValueError("state must have %d entries, got %d" % (self.X, s.size))
        self._check(self._L.mppi_update_phase1(self._h, _p(s), float(time)))
        self._rolled_out_state = s.copy()

    def update_phase2(self):
        self._check(self._L.mppi_update_phase2(self._h))

    def update_phase3(self, time):
        self._check(self._L.mppi_update_phase3(self._h))

    def device_costs_ptr(self):
        return self._L.mppi_device_costs(self._h)

    def device_gradient_ptr(self):
        return self._L.mppi_device_gradient(self._h)

    # -- queries -----------------------------------------------------------------------------
    def get(self, time, control=None):
        out = np.zeros(self.C) if control is None else control
        self._check(self._L.mppi_get(self._h, float(time), _p(out)))
        return out

    def __call__(self, time):
        return self.get(time)

    def get_state_dof(self):
        return self.X

    def get_control_dof(self):
        return self.C

    def get_time_step(self):
        return self.configuration.time_step

    def get_step_count(self):
        return self.H

    def get_update_duration(self):
        d = C.c_double()
        self._check(self._L.mppi_update_duration(self._h, C.byref(d)))
        return d.value

    def get_update_last(self):
        """Trajectory::get_update_last: the engine's own (every update entry counts)."""
        d = C.c_double()
        self._check(self._L.mppi_update_last(self._h, C.byref(d)))
        return d.value

    def get_update_count(self):
        """Trajectory::get_update_count: the engine's count of successful updates."""
        return self.update_info()["update_count"]

    def device_costs_count(self):
        """Doubles of device_costs_ptr() a phase-split caller all-reduces (R + 1)."""
        return int(self._L.mppi_device_costs_count(self._h))

    def get_rollout_count(self):
        return self.R

    def get_rolled_out_state(self):
        return self._rolled_out_state.copy()

    def _vec(self, fn, n):
        out = np.zeros(n)
        self._check(fn(self._h, _p(out)))
        return out

    def get_weights(self):
        return self._vec(self._L.mppi_weights, self.R)

    def get_gradient(self):
        """C x H (Eigen column-major) returned as an (H, C) array: row k = column k."""
        return self._vec(self._L.mppi_gradient, self.C * self.H).reshape(self.H, self.C)

    def costs(self):
        return self._vec(self._L.mppi_costs, self.R)

    def noise(self):
        return self._vec(self._L.mppi_noise, self.R * self.C * self.H).reshape(self.R, self.H, self.C)

    def get_rollouts(self):
        """[(noise (H, C), cost)] per rollout (mppi.hpp:422-424)."""
        n, c = self.noise(), self.costs()
        return [(n[r], c[r]) for r in range(self.R)]

    def get_optimal_rollout(self):
        return self._vec(self._L.mppi_optimal_control, self.C * self.H).reshape(self.H, self.C)

    trajectory = get_optimal_rollout

    def get_optimal_total_cost(self):
        d = C.c_double()
        self._check(self._L.mppi_optimal_cost(self._h, C.byref(d)))
        return d.value

    def get_optimal_terms(self):
        """The optimal rollout's seven AssistedManipulation term totals (joint limit, self collision,
        workspace, energy tank, joint velocity, trajectory, manipulability): the accumulators
        BaseTest / logger::AssistedManipulation read after filter() (mppi_optimal_terms)."""
        return self._vec(self._L.mppi_optimal_terms, 7)

    def argmin(self):
        i = C.c_int64()
        self._check(self._L.mppi_argmin(self._h, C.byref(i)))
        return i.value

    def update_info(self):
        """What the last update's rollout launch did (mppi_update_info): dict of the engine's own
        choices (cooperative kernel, folded filter(), objective in the launch, tail draws,
        sampling mode 0/1/2, rows rolled out, the step at which the fifth wave's rows moved off
        the doubled SIMD or -1, the in-launch waits that gave up in the last update - which then
        failed - and summed since create)."""
        out = np.zeros(abi.MPPI_UPDATE_INFO_N, dtype=np.int64)
        self._check(self._L.mppi_update_info(self._h, out.ctypes.data_as(C.POINTER(C.c_int64)), out.size))
        keys = ("cooperative", "folded_filter", "objective_in_launch", "tail_draws", "sampling", "rows", "handover",
                "wait_timeouts", "wait_timeouts_total", "fused_update", "graph_updates", "graph_failures",
                "update_count")
        return {k: int(v) for k, v in zip(keys, out)}

    def debug_inject(self, fault, updates=1):
        """Fault injection for the failure-detection tests (mppi_debug_inject): the next `updates`
        rollout launches carry fault bits `fault` (abi.MPPI_DEBUG_*)."""
        self._check(self._L.mppi_debug_inject(self._h, int(fault), int(updates)))

    def debug_folded_cost(self):
        """The previous update's filter() cost as the last launch folded it (mppi_debug_folded_cost;
        tests only: no pending filter() is run or waited for)."""
        v = C.c_double()
        self._check(self._L.mppi_debug_folded_cost(self._h, C.byref(v)))
        return v.value

    def smoothing_windows(self):
        """(uu, tt, start_idx) of the per-dimension SG windows (SavitzkyGolayFilter::get_windows)."""
        w = self.configuration.smoothing.window
        W = self.H + 2 * w + 1
        uu, tt = np.zeros((self.C, W)), np.zeros((self.C, W))
        st = np.zeros(self.C, dtype=np.int64)
        self._check(self._L.mppi_smoothing_windows(self._h, _p(uu), _p(tt),
                                                   st.ctypes.data_as(C.POINTER(C.c_int64))))
        return uu, tt, st

    def set_timing(self, level):
        """HIP-event timing of the update path: 0 none (default), 1 the rollout kernel alone,
        2 every phase (mppi_set_timing)."""
        self._check(self._L.mppi_set_timing(self._h, int(level)))

    def rollout_kernel_times(self):
        """The rollout launch's HIP-event times (ms) of the updates run at timing level 1 since the
        last call, oldest first (mppi_rollout_kernel_times)."""
        out = (C.c_float * 64)()
        n = C.c_int(0)
        self._check(self._L.mppi_rollout_kernel_times(self._h, out, 64, C.byref(n)))
        return list(out[:n.value])

    def kernel_times(self, wait=True, detail=False):
        """[sample, rollout, weight-reduce, optimal rollout, whole update] in ms (HIP events).
        wait=False does not wait for the overlapped optimal rollout ([3] may be an earlier one's).
        detail=True appends [5], the rollout (dynamics) kernel alone ([1] also spans the cost kernel),
        [6], the weights + gradient launch alone ([2] also spans the finish kernel; timing level
        2), and [7], the cost all-reduce ahead of it (RCCL-sharded; 0 otherwise); it implies
        wait=False."""
        if detail:
            out = (C.c_float * 8)()
            self._check(self._L.mppi_kernel_times_detail(self._h, out, 8))
            return list(out)
        out = (C.c_float * 5)()
        fn = self._L.mppi_kernel_times if wait else self._L.mppi_kernel_times_nowait
        self._check(fn(self._h, out))
        return list(out)
