"""The point mass (BASELINE configs[1]) in one launch per update (pm_fused.hip): against the
five-launch path (MPPI_PM_FUSED=0) on the same device Philox stream, and against the oracle with
the device's draws replayed in the reference's draw order (mppi.cpp:242-262)."""
import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi
from oracle import oracle as O

from helpers import assert_update_parity, replay_device_draws

pytestmark = pytest.mark.gpu

TIMES = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22]   # shifts of 5, 2, 5, 0, 5, 5 steps


def _pm(S, horison, K=20):
    conf = am.point_mass_configuration(rollouts=S, horison=horison, keep_best_rollouts=K)
    t = am.Trajectory.create(conf, am.PointMassDynamics(), am.QuadraticCost())
    assert t is not None
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    return conf, t


@pytest.mark.parametrize("S,horison", [(1024, 0.32), (1000, 0.32), (2046, 0.64), (62, 0.16), (4094, 0.08)])
def test_fused_update_equals_five_launches(S, horison, monkeypatch):
    """Noise bit for bit (draws made ahead by the previous launch's tail, kept columns shifted in),
    costs bit for bit (the same per-rollout arithmetic), weights / gradient / U* and the filter()
    cost to the gradient's summation order (per-block partials in block order against the
    weights kernel's eight splits)."""
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("MPPI_PM_FUSED", fused)
        conf, t = _pm(S, horison)
        x = np.zeros(6)
        rec = []
        for j, tm in enumerate(TIMES):
            t.update(x, tm)
            info = t.update_info()
            assert info["fused_update"] == (1 if fused == "1" else 0), info
            if fused == "1":
                assert info["sampling"] == (1 if j == 0 else 2), info   # drawn ahead from the second update
            rec.append((t.noise().copy(), t.costs().copy(), t.get_weights().copy(), t.get_gradient().copy(),
                        t.get_optimal_rollout().copy(), t.get_optimal_total_cost()))
            x = x + 0.01
        out[fused] = rec
    for j, (a, b) in enumerate(zip(out["1"], out["0"])):
        np.testing.assert_array_equal(a[0][0], b[0][0], err_msg="update %d noise" % j)
        np.testing.assert_array_equal(a[0][2:], b[0][2:], err_msg="update %d noise" % j)
        # rollout 1 = -U*, which the two paths round differently (the gradient's summation order)
        np.testing.assert_allclose(a[0][1], b[0][1], rtol=0, atol=1e-12, err_msg="update %d noise" % j)
        if j == 0:   # the same nominal (zeros): the same arithmetic on the same operands
            np.testing.assert_array_equal(a[1], b[1], err_msg="update %d costs, rollouts %s differ" %
                                          (j, np.flatnonzero(a[1] != b[1])[:8]))
        else:   # every rollout rides the shifted U*, which carries the gradient's rounding
            np.testing.assert_allclose(a[1], b[1], rtol=1e-13, atol=0, err_msg="update %d costs" % j)
        # exp(-s (c - min) / (max - min)) carries the costs' rounding, scaled by s (c - min) / (max - min)
        np.testing.assert_allclose(a[2], b[2], rtol=1e-13 if j == 0 else 1e-11, atol=1e-16, err_msg="update %d weights" % j)
        np.testing.assert_allclose(a[3], b[3], rtol=0, atol=1e-12, err_msg="update %d gradient" % j)
        np.testing.assert_allclose(a[4], b[4], rtol=0, atol=1e-12, err_msg="update %d U*" % j)
        assert abs(a[5] - b[5]) <= 1e-12 * max(1.0, abs(b[5])), (j, a[5], b[5])


@pytest.mark.parametrize("S", [1024, 130])
def test_fused_update_against_oracle(S):
    """The fused path's own draws replayed through the oracle: every update's costs, argmin,
    weights, gradient, U* and filter() cost within the parity bars (tests/helpers.py)."""
    conf, dev = _pm(S, 0.32)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    x = np.zeros(6)
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    for j, tm in enumerate(TIMES):
        costs, noise = replay_device_draws(dev, orc, x, tm, prev_costs, prev_noise, 20)
        assert dev.update_info()["fused_update"] == 1
        assert_update_parity(dev, orc, "pm fused upd %d" % j)
        prev_costs, prev_noise = costs, noise
        x = x + 0.01


def test_fused_update_all_nan_and_recovery():
    """A NaN state makes every rollout cost NaN: the fused update throws "all nan rollouts"
    (mppi.cpp:369-370) without publishing, and the next valid updates run fused again."""
    conf, t = _pm(1024, 0.32)
    x = np.zeros(6)
    t.update(x, 0.0)
    u0 = t.get_optimal_rollout().copy()
    bad = x.copy()
    bad[0] = np.nan
    with pytest.raises(am.EngineError, match="ALL_NAN"):
        t.update(bad, 0.05)
    np.testing.assert_array_equal(t.get_optimal_rollout(), u0)
    for j in (2, 3):
        t.update(x, 0.05 * j)
        info = t.update_info()
        assert info["fused_update"] == 1 and info["wait_timeouts"] == 0, info
        assert np.all(np.isfinite(t.costs()))


def test_folded_filter_cost_against_oracle():
    """filter() (mppi.cpp:450-479) of each update, left pending and folded into the next launch's
    tail (block 0, from the U* and state it copied at entry): read back as that launch left it
    (mppi_debug_folded_cost, which runs nothing) and checked against the oracle's filter() of the
    update before.  No optimal-cost read in between, so every launch folds."""
    conf, dev = _pm(1024, 0.32)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    x = np.zeros(6)
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    prev_opt = None
    for j, tm in enumerate(TIMES):
        costs, noise = replay_device_draws(dev, orc, x, tm, prev_costs, prev_noise, 20)
        info = dev.update_info()
        assert info["fused_update"] == 1 and info["folded_filter"] == (0 if j == 0 else 1), info
        if prev_opt is not None:
            folded = dev.debug_folded_cost()
            assert abs(folded - prev_opt) <= 1e-11 * max(1.0, abs(prev_opt)), (j, folded, prev_opt)
        prev_opt = orc.optimal_cost()
        prev_costs, prev_noise = costs, noise
        x = x + 0.01


@pytest.mark.parametrize("S,horison,fused", [(256, 3.0, 0), (1024, 1.28, 0), (2046, 0.64, 1), (256, 1.0, 1)])
def test_fused_update_long_horizon_against_oracle(S, horison, fused):
    """The shared point-mass step (pm_model.hpp) associates differently from the oracle:
    the state cost as fma(q2, e2, fma(q1, e1, q0 e0)) and the control cost likewise against the
    oracle's sequential sums, u * (1 / m) against u / m, and p += v dt as one fma.  Over long
    horizons (300 and 128 steps, where the rounding compounds the most) the device's draws replayed
    through the oracle still meet the parity bars of tests/helpers.py; the measured worst errors
    are printed.  At 300 and 128 steps the fused launch's LDS staging does not fit
    (pm_fused_rows), so those handles run the five launches - the same pm_model.hpp step, bit for
    bit the fused costs (test_fused_update_equals_five_launches); 2046 x 64 runs the fused launch, and
    256 x 100 the fused launch with more outputs (H C = 300) than the finisher has threads."""
    conf, dev = _pm(S, horison)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    x = np.zeros(6)
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    stats = []
    for j, tm in enumerate(TIMES[:4]):
        costs, noise = replay_device_draws(dev, orc, x, tm, prev_costs, prev_noise, 20)
        assert dev.update_info()["fused_update"] == fused
        assert_update_parity(dev, orc, "pm H=%d upd %d" % (dev.H, j), stats=stats)
        du = float(np.max(np.abs(dev.get_optimal_rollout() - orc.optimal_control())))
        stats[-1] = stats[-1] + (du,)
        prev_costs, prev_noise = costs, noise
        x = x + 0.01
    print("pm H=%d (tag, cost rel, err/Delta, (J-Jmin)/Delta, worst/allowance, U* abs):" % dev.H, stats)
