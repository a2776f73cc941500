"""CPU tests of the forecast restatement (oracle/forecast_oracle.cpp).

Pinned by the known answers of the reference's own test (src/test/case/forecast.cpp:25-98) and
by an independent numpy Kalman restatement (tests/golden/gen_golden.py: KalmanForecastNp,
np.linalg.inv gain and matrix-power horison)."""
import os

import numpy as np
import pytest

from assistedmanipulation_amd import abi
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def average_config(window=1.0, states=6):
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_AVERAGE
    c.average_states = states
    c.average_window = window
    return c


def kalman_config(order, time_step=0.005, horison=0.3):
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_KALMAN
    c.kalman_observed_states = 6
    c.kalman_order = order
    c.kalman_time_step = time_step
    c.kalman_horison = horison
    return c


def w3(x, y, z):
    return [x, y, z, 0.0, 0.0, 0.0]


def test_average_known_answers():
    """ForecastTest::test_average_forecast (forecast.cpp:62-101), assertion by assertion."""
    f = O.OracleForecast(average_config(1.0, 3))
    np.testing.assert_allclose(f.get(0.0)[:3], [0, 0, 0])
    f.observe(w3(0, 1.0, 0), 1.01)
    np.testing.assert_allclose(f.get(5.0)[:3], [0, 1.0, 0])
    f.observe(w3(0, 1.5, 0), 1.5)
    np.testing.assert_allclose(f.get(10.0)[:3], [0, 1.25, 0])
    f.observe(w3(1.0, 1.0, 1.0), 3.0)
    np.testing.assert_allclose(f.get(3.0)[:3], [1, 1, 1])
    for i in range(10):
        f.observe(w3(i, i, i), 4.5 + i * 0.05)
    np.testing.assert_allclose(f.get(3.5)[:3], [4.5, 4.5, 4.5])
    # The reference test then expects update(10.0) to keep the latest observation ((9, 9, 9)),
    # but clear_old_measurements (forecast.cpp:67-86) erases every element with time <= 9.0
    # and update_average() zeroes an empty buffer: the code, which the rollout runs, gives 0.
    f.observe_time(10.0)
    np.testing.assert_allclose(f.get(10.0)[:3], [0, 0, 0])


def test_average_ignores_the_past_and_negative_window_fails():
    f = O.OracleForecast(average_config(0.5))
    f.observe(w3(2, 0, 0), 1.0)
    f.observe(w3(4, 0, 0), 0.9)   # time < m_last: ignored (forecast.cpp:113-117)
    np.testing.assert_allclose(f.get(1.0)[:3], [2, 0, 0])
    with pytest.raises(ValueError, match="prediction window time is negative"):
        O.OracleForecast(average_config(-1.0))


def test_locf_carries_forward_until_its_horison():
    """LOCFForecast (forecast.hpp:64-140).  The reference test (forecast.cpp:25-58) builds it
    with horison = 0, so its forecast(time + 1) is zero by the code it tests; here with a
    horison the observation is carried until time + horison."""
    c = abi.mppi_forecast_config()
    c.type = abi.MPPI_FORECAST_LOCF
    c.locf_observation[:] = [1.0, 2.0, 3.0, 0, 0, 0]
    c.locf_horison = 2.0
    f = O.OracleForecast(c)
    np.testing.assert_allclose(f.get(0.0)[:3], [1, 2, 3])      # valid_until = 0 initially
    assert not f.get(0.5).any()
    rng = np.random.default_rng(0)
    for t in (0.0, 1.0, 2.5):
        w = rng.normal(size=6)
        f.observe(w, t)
        np.testing.assert_array_equal(f.get(t), w)
        np.testing.assert_array_equal(f.get(t + 2.0), w)
        assert not f.get(t + 2.0 + 1e-9).any()


@pytest.mark.parametrize("order", [1, 2])
def test_kalman_against_numpy(order):
    """Kalman filter update, derivative estimates, observe_time predictions and the sampled
    horison table against the independent numpy restatement."""
    g = np.load(os.path.join(GOLDEN, "kalman.npz"), allow_pickle=False)
    p = "o%d_" % order
    f = O.OracleForecast(kalman_config(order, float(g[p + "time_step"]), float(g[p + "horison"])))
    H, dt = int(g[p + "H"]), float(g[p + "dt"])
    tables = iter(g[p + "tables"])
    n = 0
    for ev in g[p + "events"]:
        kind, t, w = int(ev[0]), float(ev[1]), ev[2:]
        if kind == 0:
            f.observe(w, t)
        elif kind == 1:
            f.observe_time(t)
        else:
            ref = next(tables)
            got = f.table(t, dt, H)
            scale = max(1.0, np.max(np.abs(ref)))
            assert np.max(np.abs(got - ref)) <= 1e-8 * scale, (n, np.max(np.abs(got - ref)))
            n += 1
    assert n == len(g[p + "tables"])


def test_kalman_beyond_horison_is_zero():
    f = O.OracleForecast(kalman_config(1, 0.01, 0.05))
    f.observe(np.ones(6), 0.0)
    assert f.get(0.05).any()
    assert not f.get(0.0500001).any()
