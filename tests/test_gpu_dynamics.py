"""GPU parity of the device-resident FrankaRidgeback::PinocchioDynamics object (fr_object.hip via
mppi_dynamics_*), DynamicsForecast::forecast on it, and Cost::get_cost against it, with the
oracle's Pinocchio-order restatement (oracle/mppi_oracle.cpp oracle_dyn_*) as the checker.

Reference: frankaridgeback/pinocchio_dynamics.cpp:84-260 (constructor, set_state, calculate,
step), frankaridgeback/dynamics.cpp:104-138 (DynamicsForecast::forecast),
objective/assisted_manipulation.cpp:37-72 and track_point.cpp:10-34 (get_cost).
"""
import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi
from oracle import oracle as O

pytestmark = pytest.mark.gpu

# fp64 on both sides; the device solves M a = tau by CRBA + Cholesky, the oracle by Pinocchio's ABA.
# States, poses, velocities, Jacobians: 1e-10 relative.  Accelerations are M(q)^-1 tau with the
# 0.1 kg fingers in M (condition ~1e5) and arm torques of O(20): the two solves differ by up to
# ~4e-10 relative there (measured, step 27 of the stepping test), so they get 1e-8.
STATE_RTOL = 1e-10
ACC_RTOL = 1e-8
# joint velocities integrate those accelerations (qd += qdd dt): measured 1.02e-10 relative on the
# finger velocity after 38 steps, so the state's velocity half gets 1e-9
VEL_RTOL = 1e-9
# set_state's tau += NLE(q, v) at the velocities 40 random-torque steps built up: the Coriolis
# terms are quadratic in v and the sum cancels; measured 7.0e-9 relative on one joint
TAU_RTOL = 3e-8
EE = abi.MPPI_EE_N
EE_ACC = slice(abi.MPPI_EE_LINEAR_ACCELERATION, abi.MPPI_EE_ANGULAR_ACCELERATION + 3)


def _close(a, b, rtol, what):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    rtol = np.broadcast_to(np.asarray(rtol, dtype=np.float64), b.shape)
    scale = np.maximum(np.abs(b), 1.0)
    err = np.abs(a - b) / scale / rtol
    assert err.max() <= 1.0, "%s: max err %.3e of its tolerance at %d (%r vs %r)" % (
        what, err.max(), int(np.argmax(err)), a.reshape(-1)[np.argmax(err)], b.reshape(-1)[np.argmax(err)])


def _tol_state():
    t = np.full(31, STATE_RTOL)   # FrankaRidgeback's state: q, qd, tau, available energy
    t[12:24] = VEL_RTOL
    return t


def _tol_ee():
    t = np.full(EE, STATE_RTOL)
    t[abi.MPPI_EE_LINEAR_VELOCITY:abi.MPPI_EE_ANGULAR_VELOCITY + 3] = VEL_RTOL   # J qd: measured 4.6e-10
    t[EE_ACC] = ACC_RTOL
    return t


def _tol_query():
    t = np.full(abi.MPPI_DYNAMICS_QUERY_N, STATE_RTOL)
    t[12:24] = VEL_RTOL   # joint velocities
    t[24:36] = ACC_RTOL   # joint accelerations
    t[36:48] = TAU_RTOL   # torques: set_state adds NLE(q, v) to the stale torque
    return t


def _tol_rows(n):
    t = np.full(abi.MPPI_DF_N, STATE_RTOL)
    e = abi.MPPI_DF_END_EFFECTOR
    t[e + abi.MPPI_EE_LINEAR_VELOCITY:e + abi.MPPI_EE_ANGULAR_VELOCITY + 3] = VEL_RTOL
    t[abi.MPPI_DF_END_EFFECTOR + EE_ACC.start:abi.MPPI_DF_END_EFFECTOR + EE_ACC.stop] = ACC_RTOL
    return np.tile(t, (n, 1))


def _ee_close(dev_row, orc_row, what):
    # the quaternion's sign follows Eigen's branch on both sides: compared directly
    _close(dev_row, orc_row, _tol_ee(), what)


def _controls(rng, n):
    u = np.zeros((n, 12))
    u[:, 0:2] = rng.normal(0, 0.3, (n, 2))
    u[:, 2] = rng.normal(0, 0.5, n)
    u[:, 3:10] = rng.normal(0, 20.0, (n, 7))
    u[:, 10:] = rng.normal(0, 0.02, (n, 2))   # ignored by step() (only the arm's torques)
    return u


def test_object_steps_match_oracle():
    """Constructor (set_state of the initial state), 40 steps with random controls, then a
    set_state whose calculate() adds NLE onto the torque the last step left (the stale-torque
    acceleration), then more steps: state, EndEffectorState and the members."""
    x0 = am.huddled_state()
    x0[12 + 3:12 + 10] = np.linspace(-0.5, 0.5, 7)
    x0[30] = 15.0
    dev = am.PinocchioDynamicsObject.create(x0)
    orc = O.OracleDynamics(x0)
    _ee_close(dev.get_end_effector_state_row(), orc.end_effector(), "EE after create")
    _close(dev.query_row(), orc.query(), _tol_query(), "members after create")
    rng = np.random.default_rng(3)
    for k, u in enumerate(_controls(rng, 40)):
        xd, xo = dev.step(u, 0.01), orc.step(u, 0.01)
        _close(xd, xo, _tol_state(), "state step %d" % k)
        _ee_close(dev.get_end_effector_state_row(), orc.end_effector(), "EE step %d" % k)
    _close(dev.get_state(), orc.get_state(), _tol_state(), "get_state")
    x1 = dev.get_state()
    dev.set_state(x1, 0.4)
    orc.set_state(x1, 0.4)
    qd, qo = np.asarray(dev.query_row()), orc.query()
    assert np.abs(qo[24:36]).max() > 1e-3   # the stale torque accelerates the joints
    _close(qd, qo, _tol_query(), "members after set_state (stale torque)")
    _ee_close(dev.get_end_effector_state_row(), orc.end_effector(), "EE after set_state")
    for k, u in enumerate(_controls(rng, 10)):
        _close(dev.step(u, 0.01), orc.step(u, 0.01), _tol_state(), "state step %d after set_state" % k)
    ee = dev.get_end_effector_state()
    assert ee.jacobian.shape == (6, 12) and abs(np.linalg.norm(ee.orientation) - 1.0) < 1e-14
    np.testing.assert_allclose(ee.rotation @ ee.rotation.T, np.eye(3), rtol=0, atol=1e-14)


def test_dynamics_forecast_rows_match_oracle():
    """DynamicsForecast::forecast (dynamics.cpp:104-138): two consecutive forecasts of 64 steps
    (the second one starts from the torque the first left), wrench rows passed through."""
    x0 = am.huddled_state()
    x0[12 + 3:12 + 10] = np.linspace(-1.0, 1.0, 7)
    x0[30] = 5.0
    dev = am.PinocchioDynamicsObject.create(am.huddled_state())
    orc = O.OracleDynamics(am.huddled_state())
    rng = np.random.default_rng(9)
    wrench = rng.normal(0, 10, (64, 6))
    for j, t in enumerate((0.0, 0.05)):
        rd = dev.forecast_rows(x0, t, 0.01, 64, wrench)
        ro = orc.forecast_rows(x0, t, 0.01, 64, wrench)
        np.testing.assert_array_equal(rd[:, abi.MPPI_DF_WRENCH:], wrench)
        assert np.all(rd[:, abi.MPPI_DF_JOINT_POWER] == 0.0) and np.all(rd[:, abi.MPPI_DF_EXTERNAL_POWER] == 0.0)
        _close(rd, ro, _tol_rows(64), "forecast %d rows" % j)
        x0 = x0.copy()
        x0[12:24] *= -1.0


@pytest.mark.parametrize("objective", ["default", "energy", "no_forecast", "track_point"])
def test_get_cost_against_object_matches_oracle(objective):
    """Cost::get_cost(state, control, dynamics, time) on the device against the object's cached
    kinematics (the one-step lag of the reference's calculate()), and its seven terms."""
    cost = am.TrackPoint(point=(0.8, 0.6, 0.9)) if objective == "track_point" else am.AssistedManipulation()
    if objective == "track_point":
        c = cost.configuration
        c.enable_joint_limits = c.enable_self_collision_avoidance = c.enable_reach_limits = 1
    if objective == "energy":
        cost.configuration.enable_energy_limit = 1
    x0 = am.huddled_state()
    x0[30] = 15.0
    dev = am.PinocchioDynamicsObject.create(x0)
    orc = O.OracleDynamics(x0)
    rng = np.random.default_rng(4)
    wrench = None if objective == "no_forecast" else np.array([20.0, 5.0, -3.0, 0.0, 0.0, 0.0])
    for k, u in enumerate(_controls(rng, 12)):
        x = orc.step(u, 0.01)
        dev.step(u, 0.01)
        cd, td = am.evaluate_cost(cost, dev, x, u, wrench)
        co, to = orc.evaluate_cost(cost.descriptor(), x, wrench)
        assert abs(cd - co) <= 1e-11 * max(abs(co), 1.0), (k, cd, co)
        np.testing.assert_allclose(td, to, rtol=1e-10, atol=1e-9, err_msg="terms step %d" % k)
        if objective == "no_forecast":
            assert td[5] == 0.0


def test_dynamics_forecast_class_with_device_kalman():
    """The Python DynamicsForecast (dynamics.hpp:122-387) over a Trajectory's device Kalman
    forecast: the wrench rows are forecast(t + k dt) of that forecast, get_end_effector_wrench reads
    the forecast itself, parameterise keeps the reference's absolute-time horison check."""
    conf = am.frankaridgeback_configuration(rollouts=64, horison=0.16)
    traj = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    traj.attach_forecast(am.kalman_forecast_configuration(0.01, 0.5, 1))
    for i, t in enumerate(np.arange(0.0, 0.2, 0.01)):
        traj.observe_wrench(np.array([10.0 + 5 * t, 0.0, 2.0, 0.0, 0.0, 0.0]), float(t))
    df = am.DynamicsForecast(0.01, 0.3, am.PinocchioDynamicsObject.create(am.huddled_state()), traj)
    x = am.huddled_state()
    df.forecast(x, 0.2)
    assert df.get_last_forecast_time() == 0.2
    W = df.get_wrench_trajectory()
    assert W.shape == (30, 6)
    for k in (0, 7, 29):
        np.testing.assert_array_equal(W[k], traj.forecast(0.2 + k * 0.01))
    np.testing.assert_array_equal(df.get_end_effector_wrench(0.23), traj.forecast(0.23))
    assert df.parameterise(0.1) == 0 and df.parameterise(0.255) == 5 and df.parameterise(0.31) == 29
    q = df.get_joint_position()
    np.testing.assert_array_equal(q[0], x[:12])
    orc = O.OracleDynamics(am.huddled_state())
    _close(df.rows, orc.forecast_rows(x, 0.2, 0.01, 30, W), _tol_rows(30), "DynamicsForecast rows")
    assert df.get_end_effector_state(0.25).position.shape == (3,)
