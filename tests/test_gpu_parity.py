"""GPU parity: the HIP engine (through the C-ABI) against the fp64 CPU oracle on identical
injected noise.  Bar: costs within COST_RTOL of the oracle, argmin index bit-exact, weights /
gradient / U* / optimal cost within the stated tolerances (tests/helpers.py)."""
import ctypes as C

import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi
from oracle import oracle as O

from helpers import assert_update_parity, energy_only_cost, fr_pair, pm_pair, replay_device_draws, step_both

pytestmark = pytest.mark.gpu


def test_point_mass_config2():
    conf, dev, orc, sd = pm_pair(S=1024, horison=0.32)
    rng = np.random.default_rng(12345)
    x = np.zeros(6)
    for j in range(5):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "pm upd %d" % j)
        nd, no = dev.noise(), orc.noise()
        np.testing.assert_array_equal(nd[0], no[0])
        np.testing.assert_array_equal(nd[2:], no[2:])          # sampled eps: placed bit-exactly
        np.testing.assert_allclose(nd[1], no[1], rtol=0, atol=1e-12)   # rollout 1 = -U* (rounding)
        x = x + 0.01


def test_frankaridgeback_config1_compat_uint8():
    """Config 1: 128 x 32, the reference's own uint8 index semantics."""
    conf, dev, orc, sd = fr_pair(S=128, horison=0.32)
    dev.set_index_semantics(abi.MPPI_INDEX_COMPAT_UINT8)
    rng = np.random.default_rng(12345)
    x = am.huddled_state()
    for j in range(6):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "fr128 upd %d" % j)
    nd, no = dev.noise(), orc.noise()
    np.testing.assert_array_equal(nd[2:], no[2:])
    np.testing.assert_allclose(nd[1], no[1], rtol=0, atol=1e-9)


def test_frankaridgeback_config3_full_size():
    """Config 3: 4096 x 64 (wide indices), three consecutive updates (shift + keep-best)."""
    conf, dev, orc, sd = fr_pair(S=4096, horison=0.64, threads=16)
    rng = np.random.default_rng(7)
    x = am.huddled_state()
    for j in range(3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "fr4096 upd %d" % j)


def test_smoothing_savitzky_golay():
    """Config 5's SG recurrence (window 10, order 1) on a 128 x 64 problem."""
    conf, dev, orc, sd = fr_pair(S=128, horison=0.64, smoothing=am.Smoothing(10, 1))
    rng = np.random.default_rng(3)
    x = am.huddled_state()
    for j in range(5):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "sg upd %d" % j)


def test_get_interpolation_and_default():
    conf, dev, orc, sd = fr_pair(S=64, horison=0.32)
    rng = np.random.default_rng(5)
    x = am.huddled_state()
    step_both(dev, orc, x, 0.0, rng, sd)
    step_both(dev, orc, x, 0.05, rng, sd)
    for t in (0.05, 0.053, 0.071, 0.2, 0.35, 0.36, 1.0):
        np.testing.assert_allclose(dev.get(t), orc.get(t), rtol=0, atol=1e-9)
    with pytest.raises(am.EngineError):
        dev.get(0.01)   # before the last update (mppi.cpp:483 asserts)


def test_nan_rollouts_get_zero_weight():
    """Rollouts whose dynamics blow up (finite 1e300 torque noise -> inf -> NaN) get NaN costs
    and zero weight (mppi.cpp:331-334, 385-388); the next update sorts their NaN costs last
    (documented deviation: the reference's comparator is not a strict weak order with NaN)."""
    conf, dev, orc, sd = fr_pair(S=64, horison=0.16, K=8)
    rng = np.random.default_rng(11)
    x = am.huddled_state()
    step_both(dev, orc, x, 0.0, rng, sd)
    n = orc.noise_draws(0.05)
    eps = rng.standard_normal((n, 12)) * sd
    for r in (5, 9, 30):
        eps[r * 16, 4] = 1e300   # arm torque at the first column of some resampled rollouts
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    orc.update(x, 0.05)
    dev.update(x, 0.05)
    assert np.isnan(orc.costs()).sum() == 3
    assert_update_parity(dev, orc, "nan")
    assert np.all(dev.get_weights()[np.isnan(dev.costs())] == 0.0)
    for j in (2, 3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "after nan %d" % j)


@pytest.mark.parametrize("S", [4500, 20000])
def test_stable_order_at_scale(S):
    """The chunked rank (chunk sort + binary-search merge, kernels.hip) beyond one merge group
    (16 chunks of 256): the previous costs hold exact ties (the first update's kept rollouts
    duplicate rollout 0) and NaNs, so the keep-best set and every resampled rollout's draws
    (noise tensor, bit-exact) depend on the full stable order including both tie rules."""
    conf, dev, orc, sd = fr_pair(S=S, horison=0.04, K=20, threads=16)
    rng = np.random.default_rng(S)
    x = am.huddled_state()
    step_both(dev, orc, x, 0.0, rng, sd)
    n = orc.noise_draws(0.05)
    eps = rng.standard_normal((n, 12)) * sd
    for r in (7, 300, S // 2, S - 30):
        eps[r * 4, 4] = 1e300   # NaN costs at scattered resampled rollouts
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    orc.update(x, 0.05)
    dev.update(x, 0.05)
    assert np.isnan(orc.costs()).sum() == 4
    for j in (2, 3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "S=%d upd %d" % (S, j))
        np.testing.assert_array_equal(dev.noise()[2:], orc.noise()[2:])


def test_nan_noise_poisons_gradient_like_the_reference():
    """NaN eps: 0 * NaN = NaN in the gradient sum, so U* becomes NaN on both sides."""
    conf, dev, orc, sd = fr_pair(S=32, horison=0.08, K=4)
    rng = np.random.default_rng(2)
    x = am.huddled_state()
    n = orc.noise_draws(0.0)
    eps = rng.standard_normal((n, 12)) * sd
    eps[3 * 8] = np.nan
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    orc.update(x, 0.0)
    dev.update(x, 0.0)
    np.testing.assert_array_equal(np.isnan(dev.costs()), np.isnan(orc.costs()))
    np.testing.assert_array_equal(np.isnan(dev.get_optimal_rollout()), np.isnan(orc.optimal_control()))


def test_all_nan_raises():
    conf, dev, orc, sd = fr_pair(S=16, horison=0.08, K=4)
    x = am.huddled_state()
    x[12:24] = np.nan          # NaN state: every rollout's first cost is NaN
    n = orc.noise_draws(0.0)
    eps = np.zeros((n, 12))
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    with pytest.raises(RuntimeError, match="ALL_NAN"):
        orc.update(x, 0.0)
    with pytest.raises(am.EngineError, match="ALL_NAN"):
        dev.update(x, 0.0)


@pytest.mark.parametrize("S", [32, 20000])
def test_flat_costs_early_return(S):
    """All costs equal -> difference < 1e-6 -> weights / gradient left stale (mppi.cpp:373-375).
    S = 20000 takes the large-R softmin path (three launches, kernels.hip SM_LARGE_R)."""
    conf, dev, orc, sd = fr_pair(S=S, horison=0.08, K=4, threads=16)
    x = am.huddled_state()
    n = orc.noise_draws(0.0)
    dev.inject_noise(np.zeros((n, 12)))
    orc.inject_noise(np.zeros((n, 12)))
    orc.update(x, 0.0)
    dev.update(x, 0.0)
    assert np.all(dev.get_weights() == 0.0) and np.all(orc.weights() == 0.0)
    assert_update_parity(dev, orc, "flat")


def _hip():
    L = C.CDLL("libamdhip64.so.7")
    L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    L.hipDeviceSynchronize.argtypes = []
    return L


@pytest.mark.parametrize("S,hor", [(256, 0.32), (20000, 0.08)])
def test_two_shards_on_one_device_equal_unsharded(S, hor):
    """Sample sharding through the phase-split ABI: two handles on one GPU each
    own half the rollouts; the two all-reduces are done on the host.  Must equal one handle.
    S = 20000: every shard weighs all R global costs through the large-R softmin path."""
    conf, single, orc, sd = fr_pair(S=S, horison=hor)
    shards = []
    for r in range(2):
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.set_noise_source(abi.MPPI_NOISE_HOST_INJECTED)
        t.set_forecast(am.constant_forecast(t.H))
        t.set_shard(2, r)
        shards.append(t)
    hip = _hip()
    R, HC = single.R, single.H * single.C
    rng = np.random.default_rng(99)
    x = am.huddled_state()

    def allreduce(ptrs, n):
        bufs = [np.zeros(n) for _ in ptrs]
        for p, b in zip(ptrs, bufs):
            assert hip.hipMemcpy(b.ctypes.data, p, n * 8, 2) == 0   # D2H
        s = bufs[0] + bufs[1]
        for p in ptrs:
            assert hip.hipMemcpy(p, s.ctypes.data, n * 8, 1) == 0   # H2D

    for j in range(4):
        t = 0.05 * j
        n = single.noise_draws(t)
        eps = rng.standard_normal((n, 12)) * sd
        single.inject_noise(eps)
        single.update(x, t)
        for sh in shards:
            sh.inject_noise(eps)
            sh.update_phase1(x, t)
        hip.hipDeviceSynchronize()
        allreduce([sh.device_costs_ptr() for sh in shards], R + 1)   # + slot R: wait timeouts
        for sh in shards:
            sh.update_phase2()
        hip.hipDeviceSynchronize()
        allreduce([sh.device_gradient_ptr() for sh in shards], HC)
        for sh in shards:
            sh.update_phase3(t)
        for sh in shards:
            if j == 0:   # identical inputs -> per-rollout bit-exact
                np.testing.assert_array_equal(sh.costs(), single.costs())
            else:        # U* differs in the last bit (gradient summed per shard, then across)
                np.testing.assert_allclose(sh.costs(), single.costs(), rtol=1e-13, atol=0)
            np.testing.assert_allclose(sh.get_optimal_rollout(), single.get_optimal_rollout(), rtol=0, atol=1e-12)
            np.testing.assert_allclose(sh.get_weights(), single.get_weights(), rtol=0, atol=1e-15)
            assert sh.argmin() == single.argmin()


def test_philox_noise_statistics_and_replay():
    """Device Philox mode: eps ~ N(0, Sigma) per component, and replaying the device's draws
    through the oracle reproduces the update (so the device consumed them where the reference
    would have)."""
    conf = am.frankaridgeback_configuration(rollouts=2048, horison=0.32, keep_best_rollouts=20, threads=8)
    dev = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    dev.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    table = am.constant_forecast(dev.H)
    dev.set_forecast(table)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    orc.set_forecast(table)
    x = am.huddled_state()
    prev_costs = np.zeros(dev.R)
    prev_noise = np.zeros((dev.R, dev.H, dev.C))
    sd = np.sqrt(np.diag(conf.covariance))
    for j in range(3):
        t = 0.05 * j
        shift = int((t - (0.05 * (j - 1) if j > 0 else 0.0)) / conf.time_step) if j > 0 else 0
        dev.update(x, t)
        noise = dev.noise()
        if j == 0:
            z = noise[2 + 20:] / np.where(sd > 0, sd, 1.0)
            z = z[..., sd > 0].reshape(-1)
            assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
            assert np.all(noise[..., sd == 0] == 0.0)
        # reconstruct the draw stream in the reference's order (mppi.cpp:242-262)
        order = 2 + np.argsort(np.where(np.isnan(prev_costs[2:]), np.inf, prev_costs[2:]), kind="stable")
        keep_idx, res_idx = order[:20], order[20:]
        shifted = dev.H - shift
        draws = []
        if shift > 0:
            for r in keep_idx:
                draws.append(noise[r, shifted:])
                np.testing.assert_array_equal(noise[r, :shifted], prev_noise[r, shift:])
        for r in res_idx:
            draws.append(noise[r])
        orc.inject_noise(np.concatenate(draws, axis=0) if draws else np.zeros((0, 12)))
        orc.update(x, t)
        assert_update_parity(dev, orc, "philox upd %d" % j)
        prev_costs, prev_noise = dev.costs(), noise


def _track_point_all_terms(point=(0.8, 0.6, 0.9)):
    tp = am.TrackPoint(point=point)
    c = tp.configuration
    c.enable_joint_limits = c.enable_self_collision_avoidance = c.enable_reach_limits = 1
    return tp


def test_track_point_objective():
    """TrackPoint (track_point.cpp) as the device cost, every term enabled,
    starting next to two joint limits so the hard-coded limit terms fire."""
    conf, dev, orc, sd = fr_pair(S=128, horison=0.32, cost=_track_point_all_terms())
    rng = np.random.default_rng(99)
    x = am.huddled_state()
    x[3], x[6] = 2.89, 0.06
    for j in range(4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "trackpoint upd %d" % j)


def test_energy_tank_with_every_term():
    """a10.7: enable_energy_limit on top of the default cost stack (the tank's power needs the NLE,
    SURVEY §8f item 3); tank started inside its barriers."""
    cost = am.AssistedManipulation()
    cost.configuration.enable_energy_limit = 1
    conf, dev, orc, sd = fr_pair(S=128, horison=0.32, cost=cost)
    rng = np.random.default_rng(31)
    x = am.huddled_state()
    x[30] = 15.0
    for j in range(4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "energy+all upd %d" % j)


# The barriers amplify the tank's rounding: dJ/J = sum_k |c'(E_k)| E_k / J * (dE/E), and with
# c = 10/E + 10/(20 - E) a rollout that passes E = 19.995 has sum |c'(E_k)| E_k / J ~ 3.4e3
# (measured on the oracle: rollout 75 of update 1 below), so 1e-14 relative in E is 3.4e-11 in J.
ENERGY_COST_RTOL = 1e-9
ENERGY_WEIGHT_ATOL = 1e-9


@pytest.mark.parametrize("e0", [15.0, 0.3])
def test_energy_only_cost(e0):
    """The tank's barrier alone decides the weights: every rollout's energy trajectory is checked
    through its cost; E0 = 0.3 sits next to the Left(0, 10) bound and the max(0, .) clamp, and the
    state carries a velocity so NLE . v is nonzero from the first step."""
    conf, dev, orc, sd = fr_pair(S=256, horison=0.32, cost=energy_only_cost())
    rng = np.random.default_rng(32)
    x = am.huddled_state()
    x[30] = e0
    x[12 + 3:12 + 10] = rng.normal(0, 0.5, 7)
    for j in range(4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "energy-only E0=%g upd %d" % (e0, j), ENERGY_COST_RTOL, ENERGY_WEIGHT_ATOL)


@pytest.mark.parametrize("fixture", ["update_s16_h8.npz", "update_s24_h16_sg.npz", "update_s16_h8_trackpoint.npz",
                                     "update_s16_h8_energy.npz"])
def test_device_against_golden_fixtures(fixture):
    """The device path against the independent numpy restatement (tests/golden/gen_golden.py)
    directly, same injected eps: pins the kernels without going through the oracle."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", fixture), allow_pickle=False)
    S, K, H = int(g["S"]), int(g["K"]), int(g["H"])
    w, order = (int(v) for v in g["smoothing"])
    conf = am.frankaridgeback_configuration(rollouts=S, horison=H * 0.01, keep_best_rollouts=K,
                                            smoothing=am.Smoothing(w, order) if w else None)
    objective = str(g["objective"]) if "objective" in g else "assisted_manipulation"
    cost = {"track_point": lambda: _track_point_all_terms(g["track_point"]),
            "energy_only": energy_only_cost}.get(objective, am.AssistedManipulation)()
    dev = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), cost)
    dev.set_noise_source(abi.MPPI_NOISE_HOST_INJECTED)
    dev.set_forecast(g["forecast"])
    offs = np.concatenate([[0], np.cumsum(g["eps_counts"])])
    for j, t in enumerate(g["time"]):
        assert dev.noise_draws(float(t)) == g["eps_counts"][j]
        dev.inject_noise(g["eps"][offs[j]:offs[j + 1]])
        dev.update(g["x0"], float(t))
        c = dev.costs()
        np.testing.assert_allclose(c, g["costs"][j], rtol=ENERGY_COST_RTOL if objective == "energy_only" else 1e-11, atol=0)
        assert dev.argmin() == int(np.nanargmin(g["costs"][j]))
        np.testing.assert_allclose(dev.get_weights(), g["weights"][j], rtol=0, atol=1e-10)
        np.testing.assert_allclose(dev.get_gradient(), g["gradient"][j], rtol=0, atol=1e-8)
        np.testing.assert_allclose(dev.get_optimal_rollout(), g["U"][j], rtol=0, atol=1e-8)
        assert abs(dev.get_optimal_total_cost() - g["opt_cost"][j]) <= 1e-11 * abs(g["opt_cost"][j])


@pytest.mark.parametrize("rollouts,objective", [(2046, "am"), (1000, "am"), (4096, "am"), (2046, "energy"),
                                                (1000, "track_point"), (4096, "track_point")])
def test_draws_ahead_match_sampling_at_update(rollouts, objective, monkeypatch):
    """Draws made behind the previous publish (MPPI_DRAW_AHEAD, the default for device Philox) with
    the kept rollouts' columns copied in by the rollout launch equal the sampling launch at update
    time, bit for bit, over updates whose shift varies (5, 2, 5, 0 steps) with kept rollouts; for
    the default objective, the energy-tank variant (articulated-body kernel) and TrackPoint.  Both
    ways of drawing ahead: all rows behind the publish (MPPI_TAIL_DRAWS=0), and the main waves'
    rows in the rollout launch's tail with the rest behind the publish (the default; 1000 and 4096
    rollouts leave rows over, so their launches have a fifth wave and draw in the tail)."""
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=0.32, keep_best_rollouts=20, threads=8)
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17]
    make_cost = {"am": am.AssistedManipulation, "energy": energy_only_cost, "track_point": _track_point_all_terms}[objective]
    out = {}
    for ahead in ("0", "1", "tail"):
        monkeypatch.setenv("MPPI_DRAW_AHEAD", "0" if ahead == "0" else "1")
        monkeypatch.setenv("MPPI_TAIL_DRAWS", "1" if ahead == "tail" else "0")
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), make_cost())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for tm in times:
            t.update(x, tm)
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[ahead] = rec
    for mode in ("1", "tail"):
        for j, (a, b) in enumerate(zip(out["0"], out[mode])):
            for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
                np.testing.assert_array_equal(u, v, err_msg="%s: update %d %s" % (mode, j, name))


@pytest.mark.parametrize("rollouts,objective", [(4096, "am"), (4096, "energy"), (4096, "track_point"), (1000, "am"),
                                                (4097, "am")])
def test_handover_equals_doubled_simd(rollouts, objective, monkeypatch):
    """take_over (fr_coop.hip): the fifth wave's rows move, mid-horizon, to the first of waves 1..3
    to end its own rows, off the SIMD the fifth wave shares with wave 0.  The moved rows resume from
    the (q, qd, E) the fifth wave left at the top of a step, so every output equals the launch that
    keeps them on the doubled SIMD (MPPI_HANDOVER=0), bit for bit, over updates with kept rollouts
    and shifts; 1000 rollouts have fifth waves in three workgroups, 4097 four leftover rows."""
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=0.64, keep_best_rollouts=20, threads=8)
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17]
    make_cost = {"am": am.AssistedManipulation, "energy": energy_only_cost, "track_point": _track_point_all_terms}[objective]
    out, steps = {}, []
    for ho in ("0", "1"):
        monkeypatch.setenv("MPPI_HANDOVER", ho)
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), make_cost())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for tm in times:
            t.update(x, tm)
            info = t.update_info()
            assert info["wait_timeouts"] == 0, info   # no in-launch wait gave up
            if ho == "1":
                steps.append(info["handover"])
            else:
                assert info["handover"] == -1, info
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[ho] = rec + [(np.float64(t.get_optimal_total_cost()),) * 4]   # the folded filter() rows
    print("handover steps:", steps)
    assert all(0 < k < 63 for k in steps), steps
    for j, (a, b) in enumerate(zip(out["0"], out["1"])):
        for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))


@pytest.mark.parametrize("rollouts,horison,objective,window", [(4096, 0.64, "am", 0), (4096, 0.64, "energy", 0),
                                                               (4096, 0.64, "track_point", 0), (1000, 0.64, "am", 0),
                                                               (4097, 0.64, "am", 0), (4096, 0.32, "am", 0),
                                                               (8192, 1.28, "am", 10), (4096, 0.16, "am", 0)])
def test_relay_members_equal_one_workgroup(rollouts, horison, objective, window, monkeypatch):
    """The rows left over relayed through several workgroups (MPPI_RELAY_K, relay_stage: member m of
    relay group q is workgroup q + 8 m, the lanes' state and the rows' partial cost sums handed on
    through global memory under the launch's token) against the relay in one workgroup: every
    output bit for bit, over updates with kept rollouts and shifts (the kept columns each member
    copies for its own steps), three objectives, three relay groups (1000 rollouts), four rows left
    over (4097), horizons of 32 and 16 steps (fewer members fit) and configs[4]'s per-GPU share
    (8192 x 128 with the Savitzky-Golay filter: the relay rides in the split's second launch)."""
    sg = am.Smoothing(window, 1) if window else None
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8,
                                            smoothing=sg)
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17]
    make_cost = {"am": am.AssistedManipulation, "energy": energy_only_cost, "track_point": _track_point_all_terms}[objective]
    out = {}
    for k in ("1", "2", "4"):
        monkeypatch.setenv("MPPI_RELAY_K", k)
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), make_cost())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for tm in times:
            t.update(x, tm)
            assert t.update_info()["wait_timeouts"] == 0
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[k] = rec + [(np.float64(t.get_optimal_total_cost()),) * 4]   # the folded filter() rows
    for k in ("2", "4"):
        for j, (a, b) in enumerate(zip(out["1"], out[k])):
            for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
                np.testing.assert_array_equal(u, v, err_msg="K=%s update %d %s" % (k, j, name))


@pytest.mark.parametrize("k", ["1", "2"])
def test_relay_kept_rows_against_oracle(k, monkeypatch):
    """The relay rows' kept columns (keep-best rollouts among the rows left over, shifted in by the
    relay's wave 4 at entry) against the oracle with the device's draws replayed, over a state change
    and shifts of 5, 2, 5, 0 and 5 steps, relay in one workgroup and over two.  A stage past the
    first issues its first eps loads before it waits for the previous stage; before it also waited
    for the kept copy (LF_KEPT_X), the one-workgroup relay read a kept rollout's unshifted eps at a
    stage's first step (rollout 1000 at update 6: 7.2e-8 of Delta, r06)."""
    monkeypatch.setenv("MPPI_RELAY_K", k)
    conf = am.frankaridgeback_configuration(rollouts=1000, horison=0.64, keep_best_rollouts=20, threads=8)
    dyn, cost = am.FrankaRidgebackDynamics(), am.AssistedManipulation()
    dev = am.Trajectory.create(conf, dyn, cost)
    dev.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    table = am.constant_forecast(dev.H)
    dev.set_forecast(table)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dyn.descriptor(), cost.descriptor(), scalar=0, mode=0)
    orc.set_forecast(table)
    x = am.huddled_state()
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    for j, t in enumerate([0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22, 0.27]):
        if j == 5:
            x = x.copy()
            x[12 + 4] = 0.3
        prev_costs, prev_noise = replay_device_draws(dev, orc, x, t, prev_costs, prev_noise, 20)
        assert dev.update_info()["wait_timeouts"] == 0
        assert_update_parity(dev, orc, "relay K=%s upd %d" % (k, j))


def test_two_philox_shards_draw_ahead_equal_unsharded():
    """Device Philox across two shards on one GPU (phase-split ABI, host all-reduces): each shard
    holds 4098 rollouts, so its rollout launch runs one round of workgroups and its draws are made
    ahead; S = 8194 > RANK_TILED_MAX, so the rank takes the chunk + merge path before those draws.
    The unsharded handle (8196 rollouts) samples at update time.  Draws are indexed by (rollout,
    step): the noise is identical, the costs too, U* to the gradient's summation order."""
    conf = am.frankaridgeback_configuration(rollouts=8194, horison=0.08, keep_best_rollouts=20, threads=8)
    mk = lambda: am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    single, shards = mk(), [mk(), mk()]
    for r, t in enumerate([single] + shards):
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        if t is not single:
            t.set_shard(2, r - 1)
    hip = _hip()
    R, HC = single.R, single.H * single.C
    x = am.huddled_state()

    def allreduce(ptrs, n):
        bufs = [np.zeros(n) for _ in ptrs]
        for p, b in zip(ptrs, bufs):
            assert hip.hipMemcpy(b.ctypes.data, p, n * 8, 2) == 0   # D2H
        s = bufs[0] + bufs[1]
        for p in ptrs:
            assert hip.hipMemcpy(p, s.ctypes.data, n * 8, 1) == 0   # H2D

    for j in range(4):
        t = 0.05 * j
        single.update(x, t)
        for sh in shards:
            sh.update_phase1(x, t)
        hip.hipDeviceSynchronize()
        allreduce([sh.device_costs_ptr() for sh in shards], R + 1)   # + slot R: wait timeouts
        for sh in shards:
            sh.update_phase2()
        hip.hipDeviceSynchronize()
        allreduce([sh.device_gradient_ptr() for sh in shards], HC)
        for sh in shards:
            sh.update_phase3(t)
        full = single.noise()
        for r, sh in enumerate(shards):   # a shard's noise() holds its rows at their global indices
            b, e = am.shard_range(R, 2, r)
            mine, ref = sh.noise()[b:e], full[b:e]
            d = max(2 - b, 0)   # rollout 1 carries -U*, which differs in the last bits (gradient order)
            np.testing.assert_array_equal(mine[d:], ref[d:], err_msg="update %d shard %d noise" % (j, r))
            np.testing.assert_allclose(mine[:d], ref[:d], rtol=0, atol=1e-12)
        for sh in shards:
            np.testing.assert_allclose(sh.costs(), single.costs(), rtol=1e-13, atol=0)
            np.testing.assert_allclose(sh.get_optimal_rollout(), single.get_optimal_rollout(), rtol=0, atol=1e-12)
            assert sh.argmin() == single.argmin()


@pytest.mark.parametrize("S", [4096, 1000])
def test_rollout_kernel_event_ring(S):
    """Timing level 1 records the rollout launch's events into a ring read after the loop
    (mppi_rollout_kernel_times): one positive time per timed update, oldest first, the record
    cleared by the read; kernel_times(detail)[5] still gives the newest; timing leaves U* alone."""
    def run(timed):
        conf = am.frankaridgeback_configuration(rollouts=S, horison=0.64, keep_best_rollouts=20)
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=11)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        assert t.rollout_kernel_times() == []
        for j in range(7):
            if timed and j % 2 == 1:
                t.set_timing(1)
            t.update(x, 0.05 * j)
            t.set_timing(0)
        t.synchronize()
        return t, t.get_optimal_rollout()
    t, u_timed = run(True)
    newest = t.kernel_times(detail=True)[5]
    times = t.rollout_kernel_times()
    assert len(times) == 3 and all(0.0 < v < 100.0 for v in times)
    assert newest == pytest.approx(times[-1])
    assert t.rollout_kernel_times() == []
    _, u_plain = run(False)
    np.testing.assert_array_equal(u_timed, u_plain)


@pytest.mark.parametrize("barriers", ["no_self_collision", "none"])
def test_default_stack_without_self_collision_4096(barriers):
    """The bench's kernel path (cooperative CRBA + Gauss-Jordan solve, objective in the launch) at
    4096 x 64 without the constant self-collision term (1.28e13 per rollout).
    "no_self_collision": the other terms stay; from the huddled state every rollout still breaches
    a joint-limit / workspace barrier on some steps (1e10 each, measured minimum 7e10), so the costs
    count breaches.  "none": every barrier off (joint, self-collision, workspace, energy), leaving
    the smooth velocity / trajectory / manipulability terms, so the relative cost bar measures the
    dynamics and kinematics alone."""
    cost = am.AssistedManipulation()
    c = cost.configuration
    c.enable_self_collision_limit = 0
    if barriers == "none":
        c.enable_joint_limit = c.enable_workspace_limit = c.enable_energy_limit = 0
    conf, dev, orc, sd = fr_pair(S=4096, horison=0.64, threads=16, cost=cost)
    rng = np.random.default_rng(7)
    x = am.huddled_state()
    stats = []
    # "none" leaves only the smooth terms, so the relative bar sees the 64-step dynamics' rounding
    # amplified: 5.7e-12 / 9.6e-12 / 6.1e-12 over three updates with the generic FK scan (r04b),
    # 7.6e-12 / 7.8e-12 / 1.1e-11 with its planar last level (r04i).  5e-11, as the 65536 x 128 case's
    # 1e-10; the north star's bar is an fp32 tolerance, and the Delta-relative bar stays at 1e-11.
    rtol = 5e-11 if barriers == "none" else 1e-11
    for j in range(3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "%s upd %d" % (barriers, j), stats=stats, cost_rtol=rtol)
        assert dev.update_info()["objective_in_launch"] == 1
        co = orc.costs()
        # no 1.28e13 floor under every rollout (barrier breaches still reach 2.75e12 on some)
        assert np.nanmin(co) < 1e12 and (barriers != "none" or np.nanmax(co) < 1e9), (np.nanmin(co), np.nanmax(co))
        if barriers == "none":
            assert np.nanmax(co) - np.nanmin(co) > 0.0
    print("cost errors (rel, /Delta, (J-Jmin)/Delta):", stats)


def test_non_diagonal_covariance_philox():
    """A non-diagonal Sigma (Gaussian::set_covariance's eigen-transform, gaussian.hpp:48-55): the
    device's full-transform Philox path (sample_kernel, T z with the engine's Jacobi T) has the
    configured covariance, and replaying its draws through the oracle reproduces the updates."""
    conf = am.frankaridgeback_configuration(rollouts=2048, horison=0.32, keep_best_rollouts=20, threads=16)
    sd = np.sqrt(am.config.FR_VARIANCE)
    corr = np.eye(12)
    for a, b, r in ((0, 1, 0.5), (3, 4, -0.4), (5, 7, 0.3), (2, 9, 0.2)):
        corr[a, b] = corr[b, a] = r
    conf.covariance = corr * np.outer(sd, sd)
    dev = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    dev.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0xC0FFEE)
    table = am.constant_forecast(dev.H)
    dev.set_forecast(table)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    orc.set_threads(16)
    orc.set_forecast(table)
    x = am.huddled_state()
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    for j in range(3):
        costs, noise = replay_device_draws(dev, orc, x, 0.05 * j, prev_costs, prev_noise, 20)
        assert dev.update_info()["sampling"] == 0   # the full transform samples at update time
        if j == 0:
            e = noise[22:].reshape(-1, 12)   # 2026 x 32 fresh draws (the first update keeps zeros)
            assert np.all(e[:, 10:] == 0.0)
            cov = np.cov(e[:, :10].T)
            np.testing.assert_allclose(np.diag(cov), sd[:10] ** 2, rtol=0.03)
            s10 = np.sqrt(np.diag(cov))
            np.testing.assert_allclose(cov / np.outer(s10, s10), corr[:10, :10], rtol=0, atol=0.03)
        assert_update_parity(dev, orc, "non-diag upd %d" % j)
        prev_costs, prev_noise = costs, noise


def test_valid_update_after_all_nan_failure():
    """An update that throws "all nan rollouts" (the reference throws without counting it,
    mppi.cpp:369-370) followed by valid updates: each later update waits for its own publish (the
    flag's sequence is per call) and matches the oracle."""
    conf, dev, orc, sd = fr_pair(S=256, horison=0.16, K=8)
    rng = np.random.default_rng(4)
    x = am.huddled_state()
    step_both(dev, orc, x, 0.0, rng, sd)
    assert_update_parity(dev, orc, "before")
    bad = x.copy()
    bad[12:24] = np.nan
    n = orc.noise_draws(0.05)
    eps = rng.standard_normal((n, 12)) * sd
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    with pytest.raises(RuntimeError, match="ALL_NAN"):
        orc.update(bad, 0.05)
    with pytest.raises(am.EngineError, match="ALL_NAN"):
        dev.update(bad, 0.05)
    for j in (2, 3, 4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert_update_parity(dev, orc, "after failure %d" % j)


@pytest.mark.parametrize("energy", [False, True])
def test_optimal_rollout_term_totals(energy):
    """mppi_optimal_terms: the optimal rollout's per-term totals that BaseTest and
    logger::AssistedManipulation read after filter() (base.cpp:140-146, logging/
    assisted_manipulation.cpp:61-90) against the oracle's accumulators; with gamma = 1 they sum
    to the optimal cost."""
    cost = am.AssistedManipulation()
    cost.configuration.enable_energy_limit = int(energy)
    conf, dev, orc, sd = fr_pair(S=256, horison=0.32, cost=cost)
    rng = np.random.default_rng(21)
    x = am.huddled_state()
    x[30] = 15.0
    assert np.all(dev.get_optimal_terms() == 0.0)   # before the first update: reset(0)
    for j in range(3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        td, to = dev.get_optimal_terms(), orc.optimal_terms()
        np.testing.assert_allclose(td, to, rtol=1e-11, atol=1e-9, err_msg="update %d" % j)
        assert (td[3] != 0.0) == energy and td[1] > 0.0
        assert abs(td.sum() - dev.get_optimal_total_cost()) <= 1e-12 * abs(dev.get_optimal_total_cost())
        assert_update_parity(dev, orc, "terms upd %d" % j)


def test_in_launch_wait_timeout_fails_the_update():
    """A bounded in-launch wait that gives up (fr_coop.hip: relay stage 1 never signals stage 2,
    injected with mppi_debug_inject) leaves the relay rows' costs unwritten, so the update fails
    with MPPI_ERR_DEVICE and publishes nothing, as the reference refuses to go on when optimise()
    throws (mppi.cpp:369-370).  The oracle cannot lose rows, so its side of the failed update is an
    all-NaN failure at the same time with the same noise: both leave U* unpublished, no filter(),
    and the same shift.  The next sample() sorts the failed update's costs (the keep-best set and
    the injected stream's order, mppi.cpp:222-262), which differ - the device's are real where the
    oracle's are NaN - so the oracle takes the device's (oracle_set_costs); the updates after the
    failure must then match the oracle again."""
    conf, dev, orc, sd = fr_pair(S=4096, horison=0.64, K=20, threads=16)
    rng = np.random.default_rng(31)
    x = am.huddled_state()
    step_both(dev, orc, x, 0.0, rng, sd)
    assert_update_parity(dev, orc, "before", check_optimal=False)
    u_before = dev.get_optimal_rollout().copy()
    n = orc.noise_draws(0.05)
    eps = rng.standard_normal((n, 12)) * sd
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    bad = x.copy()
    bad[12:24] = np.nan
    with pytest.raises(RuntimeError, match="ALL_NAN"):
        orc.update(bad, 0.05)
    dev.debug_inject(abi.MPPI_DEBUG_RELAY_NO_SIGNAL, 1)
    with pytest.raises(am.EngineError, match="wait timed out"):
        dev.update(x, 0.05)
    info = dev.update_info()
    assert info["wait_timeouts"] > 0 and info["wait_timeouts_total"] == info["wait_timeouts"], info
    np.testing.assert_array_equal(dev.get_optimal_rollout(), u_before)   # nothing published
    orc.set_costs(dev.costs())
    for j in (2, 3, 4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert dev.update_info()["wait_timeouts"] == 0
        assert_update_parity(dev, orc, "after timeout %d" % j)


def test_wait_timeout_on_one_shard_fails_every_shard():
    """Phase-split shards (an external communicator's view): the caller all-reduces the
    R + 1 doubles of mppi_device_costs, slot R being each rank's in-launch wait timeouts.  A relay
    stage of shard 0 that never signals (mppi_debug_inject) loses shard 0's relay rows, so both
    shards fail the update with MPPI_ERR_DEVICE - shard 1 from the all-reduced count alone - and
    both publish nothing; the next update succeeds on both with no timeout."""
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.32, keep_best_rollouts=20, threads=8)
    shards = []
    for r in range(2):
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=7)
        t.set_forecast(am.constant_forecast(t.H))
        t.set_shard(2, r)
        shards.append(t)
    hip = _hip()
    R, HC = shards[0].R, shards[0].H * shards[0].C
    x = am.huddled_state()

    def allreduce(ptrs, n):
        bufs = [np.zeros(n) for _ in ptrs]
        for p, b in zip(ptrs, bufs):
            assert hip.hipMemcpy(b.ctypes.data, p, n * 8, 2) == 0   # D2H
        s = bufs[0] + bufs[1]
        for p in ptrs:
            assert hip.hipMemcpy(p, s.ctypes.data, n * 8, 1) == 0   # H2D
        return s

    def update(t, expect_fail):
        for sh in shards:
            sh.update_phase1(x, t)
        hip.hipDeviceSynchronize()
        s = allreduce([sh.device_costs_ptr() for sh in shards], R + 1)
        for sh in shards:
            sh.update_phase2()
        hip.hipDeviceSynchronize()
        allreduce([sh.device_gradient_ptr() for sh in shards], HC)
        for sh in shards:
            if expect_fail:
                with pytest.raises(am.EngineError, match="wait timed out"):
                    sh.update_phase3(t)
            else:
                sh.update_phase3(t)
        return s[R]

    assert update(0.0, False) == 0.0
    u0 = [sh.get_optimal_rollout().copy() for sh in shards]
    np.testing.assert_array_equal(u0[0], u0[1])
    shards[0].debug_inject(abi.MPPI_DEBUG_RELAY_NO_SIGNAL, 1)
    assert update(0.05, True) > 0   # shard 0's lost rows, counted in slot R
    for sh, u in zip(shards, u0):
        np.testing.assert_array_equal(sh.get_optimal_rollout(), u)   # nothing published
    assert update(0.10, False) == 0.0
    np.testing.assert_array_equal(shards[0].get_optimal_rollout(), shards[1].get_optimal_rollout())


def test_folded_filter_row_against_oracle():
    """The previous update's filter() as one more row of the rollout launch (fr_coop_x_kernel's
    folded row, MPPI_INFO_FOLDED_FILTER): read back as the launch left it (mppi_debug_folded_cost,
    which runs nothing) and checked against the oracle's filter() of the update before, at 1000
    rollouts (rows left over, so the row rides along).  No optimal-cost read in between."""
    conf, dev, orc, sd = fr_pair(S=1000, horison=0.64)
    rng = np.random.default_rng(3)
    x = am.huddled_state()
    prev_opt = None
    for j in range(4):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        info = dev.update_info()
        assert info["folded_filter"] == (0 if j == 0 else 1), info
        if prev_opt is not None:
            folded = dev.debug_folded_cost()
            assert abs(folded - prev_opt) <= 1e-11 * max(1.0, abs(prev_opt)), (j, folded, prev_opt)
        prev_opt = orc.optimal_cost()
