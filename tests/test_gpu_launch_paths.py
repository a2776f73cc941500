"""The rollout launch's alternative paths give the same results (fr_coop.hip).

- The objective in chunks beside the horizon loops (cost_work, the default) against the separate
  fr_step_cost_kernel (MPPI_COSTS_IN_LAUNCH=0): both evaluate every step cost with the same code
  and sum each rollout's costs in step order (mppi.cpp:322-337), so costs, weights and U* are
  bit-identical, for the default objective, the energy-tank variant and TrackPoint, with and
  without rows left over (4096 rollouts: a relay; 4094: none, the four-wave launch), and past one
  round (20000: one-wave workgroups, each evaluating its own rows after its loop).
- A horizon past the launch's step-cost buffer (HC_MAX = 128 steps) moves the objective to
  fr_step_cost_kernel: parity against the oracle at 100 x 136.
- Rows just past two waves per SIMD (R = S + 2 at S = 8192, configs[4]'s share per GPU) run as
  two fr_coop_x_kernel launches (fr_coop_update_split) instead of one-wave workgroups whose last
  wave runs alone (MPPI_SPLIT=0): bit-identical noise, costs, U*, weights and filter() cost.
"""
import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi

from helpers import assert_update_parity, energy_only_cost, fr_pair, step_both
from test_gpu_parity import _track_point_all_terms

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rollouts,objective", [(4096, "am"), (4094, "am"), (1000, "energy"), (1000, "track_point"),
                                                (20000, "am"), (20000, "energy")])
def test_objective_in_launch_equals_cost_kernel(rollouts, objective, monkeypatch):
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=0.64, keep_best_rollouts=20, threads=8)
    make_cost = {"am": am.AssistedManipulation, "energy": energy_only_cost, "track_point": _track_point_all_terms}[objective]
    times = [0.0, 0.05, 0.07, 0.12, 0.17]
    out = {}
    for cil in ("0", "1"):
        monkeypatch.setenv("MPPI_COSTS_IN_LAUNCH", cil)
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), make_cost())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for tm in times:
            t.update(x, tm)
            info = t.update_info()
            assert info["objective_in_launch"] == int(cil), info
            assert info["wait_timeouts"] == 0, info
            rec.append((t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[cil] = rec + [(np.float64(t.get_optimal_total_cost()),) * 3]   # the folded filter() row
    for j, (a, b) in enumerate(zip(out["0"], out["1"])):
        for name, u, v in zip(("costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))


def test_long_horizon_objective_outside_launch():
    conf, dev, orc, sd = fr_pair(S=100, horison=1.36)
    assert dev.H == 136
    rng = np.random.default_rng(31)
    x = am.huddled_state()
    for j in range(3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert dev.update_info()["objective_in_launch"] == 0
        assert_update_parity(dev, orc, "H136 upd %d" % j)


@pytest.mark.parametrize("rollouts,horison,window", [(8192, 0.64, 0), (8192, 1.28, 10), (8200, 0.32, 0)])
def test_split_launch_equals_one_wave_launch(rollouts, horison, window, monkeypatch):
    """The two-launch split against the one-wave launch: the same dynamics code (coop_rows), the
    objective's step costs summed in step order by both (cost_work / fr_step_cost_kernel), draws
    ahead against sampling at update time (bit-identical by construction, test_gpu_parity), the
    min / max from the objective's atomics against a pass (exact).  Device Philox, keep-best 20,
    shifts of 5, 2, 5 and 0 steps; 8192 x 128 with the Savitzky-Golay filter is configs[4]'s share
    per GPU."""
    sg = am.Smoothing(window, 1) if window else None
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8,
                                            smoothing=sg)
    times = [0.0, 0.05, 0.07, 0.12, 0.12]
    out = {}
    for split in ("0", "1"):
        monkeypatch.setenv("MPPI_SPLIT", split)
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for j, tm in enumerate(times):
            t.update(x, tm)
            info = t.update_info()
            assert info["wait_timeouts"] == 0, info
            if split == "1":
                assert info["objective_in_launch"] == 1, info
                if j > 0:   # drawn ahead; the previous filter() rides in the second launch's relay
                    assert info["sampling"] == 2 and info["tail_draws"] == 1 and info["folded_filter"] == 1, info
            else:
                assert info["sampling"] == 0 and info["folded_filter"] == 0, info   # one-wave workgroups
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[split] = rec + [(np.float64(t.get_optimal_total_cost()),) * 4]
    for j, (a, b) in enumerate(zip(out["0"], out["1"])):
        for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))

