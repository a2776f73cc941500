"""GPU tests of the device wrench forecast (forecast.hip) through the C-ABI:
the Kalman filter kernel and the per-update forecast sampling against the oracle restatement
(oracle/forecast_oracle.cpp, itself pinned by tests/test_forecast_cpu.py) and the numpy golden
tables, and full updates with the forecast on the device against the oracle fed the same
forecast as a table."""
import os

import numpy as np
import pytest

import assistedmanipulation_amd as am
from oracle import oracle as O

from helpers import assert_update_parity, fr_pair, step_both

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# Gauss-Jordan (device) vs LU (oracle) inverse in the gain, different summation orders: the
# oracle and the numpy restatement agree to 2e-15 relative; the device is held to 1e-11.
FORECAST_RTOL = 1e-11


def _device(S=32, horison=0.32):
    conf = am.frankaridgeback_configuration(rollouts=S, horison=horison)
    dev = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    assert dev is not None
    return dev


@pytest.mark.parametrize("order", [1, 2])
def test_kalman_forecast_against_golden_and_oracle(order):
    g = np.load(os.path.join(GOLDEN, "kalman.npz"), allow_pickle=False)
    p = "o%d_" % order
    cfg = am.kalman_forecast_configuration(float(g[p + "time_step"]), float(g[p + "horison"]), order)
    dev = _device()
    dev.attach_forecast(cfg)
    orc = O.OracleForecast(cfg)
    H, dt = int(g[p + "H"]), float(g[p + "dt"])
    tables = iter(g[p + "tables"])
    for ev in g[p + "events"]:
        kind, t, w = int(ev[0]), float(ev[1]), ev[2:]
        if kind == 0:
            dev.observe_wrench(w, t)
            orc.observe(w, t)
        elif kind == 1:
            dev.observe_time(t)
            orc.observe_time(t)
        else:
            ref = next(tables)
            got = np.array([dev.forecast(t + k * dt) for k in range(H)])
            scale = max(1.0, np.max(np.abs(ref)))
            assert np.max(np.abs(got - ref)) <= FORECAST_RTOL * scale
            assert np.max(np.abs(got - orc.table(t, dt, H))) <= FORECAST_RTOL * scale


def test_locf_and_average_on_device():
    dev = _device()
    dev.attach_forecast(am.average_forecast_configuration(1.0))
    orc = O.OracleForecast(am.average_forecast_configuration(1.0))
    rng = np.random.default_rng(3)
    for i, t in enumerate((1.01, 1.5, 3.0, 4.5, 4.55, 4.6, 5.8)):
        w = rng.normal(size=6)
        dev.observe_wrench(w, t)
        orc.observe(w, t)
        np.testing.assert_array_equal(dev.forecast(t + 0.3), orc.get(t + 0.3))
    dev.observe_time(10.0)
    orc.observe_time(10.0)
    np.testing.assert_array_equal(dev.forecast(10.0), orc.get(10.0))
    dev.attach_forecast(am.locf_forecast_configuration([1, 2, 3, 0, 0, 0], horison=0.5))
    np.testing.assert_array_equal(dev.forecast(0.0), [1, 2, 3, 0, 0, 0])
    w = rng.normal(size=6)
    dev.observe_wrench(w, 2.0)
    np.testing.assert_array_equal(dev.forecast(2.5), w)
    assert not dev.forecast(2.5 + 1e-9).any()


def test_updates_with_device_kalman_forecast():
    """Full 128 x 32 updates, the trajectory cost driven by the device Kalman forecast (order 2)
    observed between updates like the actor does (actor.cpp:155-197); the oracle samples its own
    restated forecast into the table the reference's cost would query."""
    cfg = am.kalman_forecast_configuration(0.005, 0.3, 2)
    conf, dev, orc, sd = fr_pair(S=128, horison=0.32, forecast=False)
    dev.attach_forecast(cfg)
    fc = O.OracleForecast(cfg)
    rng = np.random.default_rng(17)
    x = am.huddled_state()
    obs_t = 0.0
    for j in range(6):
        t = 0.05 * j
        while obs_t <= t + 1e-12:   # a wrench every 5 ms, time ticks at 1 ms
            w = np.array([20 + 10 * np.sin(3 * obs_t), 5 * np.cos(obs_t), 2.0, 0.1, 0.0, -0.1]) + rng.normal(0, 0.5, 6)
            dev.observe_wrench(w, obs_t)
            fc.observe(w, obs_t)
            for q in (0.001, 0.002, 0.003, 0.004):
                dev.observe_time(obs_t + q)
                fc.observe_time(obs_t + q)
            obs_t += 0.005
        orc.set_forecast(fc.table(t, conf.time_step, dev.H))
        step_both(dev, orc, x, t, rng, sd)
        assert_update_parity(dev, orc, "kalman-forecast upd %d" % j)
