"""optimise() and finish() inside the rollout launch (fr_coop.hip epilogue) against the three
launches they replace (weights_gradient_kernel, finish_flat_kernel; MPPI_EPILOGUE=0): the epilogue
runs those kernels' arithmetic in the same order, so every output is bit-identical.  Device Philox
(the epilogue needs the draws made ahead), keep-best 20, shifts of 5, 2, 5, 0 and 5 steps."""
import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi

from helpers import energy_only_cost
from test_gpu_parity import _track_point_all_terms

pytestmark = pytest.mark.gpu

TIMES = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17]


def _run(rollouts, horison, make_cost, bounded=False):
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), make_cost())
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    x = am.huddled_state()
    rec, flags = [], []
    for j, tm in enumerate(TIMES):
        if j == 4:
            x = x.copy()
            x[12 + 5] = 0.4
        t.update(x, tm)
        info = t.update_info()
        assert info["wait_timeouts"] == 0, info
        flags.append(info["fused_update"])
        rec.append((t.noise().copy(), t.costs().copy(), t.get_weights().copy(), t.get_gradient().copy(),
                    t.get_optimal_rollout().copy()))
    rec.append((np.float64(t.get_optimal_total_cost()),) * 5)
    return rec, flags


@pytest.mark.parametrize("rollouts,horison,objective", [(4096, 0.64, "am"), (1000, 0.64, "am"), (4097, 0.32, "am"),
                                                        (2000, 0.64, "energy"), (1000, 0.64, "track_point")])
def test_epilogue_equals_three_launches(rollouts, horison, objective, monkeypatch):
    make_cost = {"am": am.AssistedManipulation, "energy": energy_only_cost, "track_point": _track_point_all_terms}[objective]
    out = {}
    for ep in ("0", "1"):
        monkeypatch.setenv("MPPI_EPILOGUE", ep)
        out[ep] = _run(rollouts, horison, make_cost)
    assert out["0"][1] == [0] * len(TIMES)
    assert out["1"][1] == [0] + [1] * (len(TIMES) - 1), out["1"][1]   # from the first update drawn ahead
    for j, (a, b) in enumerate(zip(out["0"][0], out["1"][0])):
        for name, u, v in zip(("noise", "costs", "weights", "gradient", "U*"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))


def test_epilogue_wait_timeout_fails_the_update(monkeypatch):
    """A relay stage that never signals (mppi_debug_inject) in a launch with the epilogue: the
    finisher sees the in-launch timeouts, publishes nothing and the update fails; the updates after
    it run the epilogue again and time nothing out."""
    monkeypatch.setenv("MPPI_EPILOGUE", "1")   # opt-in (engine.cpp epilogue_wanted)
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.64, keep_best_rollouts=20, threads=8)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    x = am.huddled_state()
    t.update(x, 0.0)
    t.update(x, 0.05)
    assert t.update_info()["fused_update"] == 1
    u = t.get_optimal_rollout().copy()
    t.debug_inject(abi.MPPI_DEBUG_RELAY_NO_SIGNAL, 1)
    with pytest.raises(am.EngineError, match="wait timed out"):
        t.update(x, 0.10)
    np.testing.assert_array_equal(t.get_optimal_rollout(), u)
    for j in (3, 4, 5):
        t.update(x, 0.05 * j)
        info = t.update_info()
        assert info["wait_timeouts"] == 0, info
        assert np.all(np.isfinite(t.get_optimal_rollout()))
    assert t.update_info()["fused_update"] == 1
