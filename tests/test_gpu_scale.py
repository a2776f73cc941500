"""GPU parity at BASELINE.json's larger workloads, on one GPU, and in the bench's own mode.

- the bench's exact mode at configs[2] (4096 x 64): device Philox, the next update's draws made
  ahead (tail draws in the rollout launch + rank_draw_kernel behind the publish), the objective
  in the launch, the previous filter() folded in as a row, keep-best 20, t = 0.05 j; the device's
  draws are replayed through the oracle (reference draw order, mppi.cpp:242-262);
- configs[3]'s total (32768 x 64) on one handle against the oracle, and as eight shards of the
  phase-split ABI (host all-reduces) against the unsharded handle;
- configs[4]'s per-GPU (8192 x 128) and total (65536 x 128) workloads with the Savitzky-Golay
  filter (window 10, order 1) against the oracle (mppi.cpp:344-448, filter.cpp:35-110).
Past one round of workgroups the engine switches paths (the two-launch split, one-wave workgroups,
the large-R softmin launches, the chunk + merge rank, sg_finish_kernel's LDS windows at H = 128):
these sizes are where those run.  The oracle runs with 16 threads (the GPU box's CPU share).
"""
import ctypes as C

import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi
from oracle import oracle as O

from helpers import assert_update_parity, fr_pair, replay_device_draws, step_both

pytestmark = pytest.mark.gpu

THREADS = 16


def test_bench_mode_replay_4096x64():
    """bench.py's update loop exactly (configs[2]), checked against the oracle on the device's own
    draws for four updates; the launch-mode flags show the bench's path was the one taken."""
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.64, keep_best_rollouts=20, threads=THREADS)
    dev = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    dev.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    table = am.constant_forecast(dev.H)
    dev.set_forecast(table)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dev.dynamics.descriptor(), dev.cost.descriptor())
    orc.set_forecast(table)
    x = am.huddled_state()
    prev_costs, prev_noise = np.zeros(dev.R), np.zeros((dev.R, dev.H, dev.C))
    stats = []
    for j in range(4):
        costs, noise = replay_device_draws(dev, orc, x, 0.05 * j, prev_costs, prev_noise, 20)
        info = dev.update_info()
        assert info["cooperative"] == 1 and info["objective_in_launch"] == 1
        if j > 0:   # drawn ahead behind the previous publish + in the previous launch's tail
            assert info["sampling"] == 2 and info["tail_draws"] == 1 and info["folded_filter"] == 1, info
        # the optimal cost is not read between updates (reading it would run filter() by itself
        # and the next launch would not fold it, as bench.py's loop does)
        assert_update_parity(dev, orc, "bench mode upd %d" % j, stats=stats, check_optimal=(j == 3))
        prev_costs, prev_noise = costs, noise
    print("cost errors (rel, /Delta, (J-Jmin)/Delta):", stats)


def test_config3_total_unsharded_32768x64():
    """configs[3]'s 32768 x 64 on one handle: one-wave workgroups (each evaluating its own rows'
    objective after its loop), the large-R softmin (R > 16384) and the chunk + merge rank (S > 8192)."""
    conf, dev, orc, sd = fr_pair(S=32768, horison=0.64, threads=THREADS)
    rng = np.random.default_rng(33)
    x = am.huddled_state()
    stats = []
    for j in range(3):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        assert dev.update_info()["objective_in_launch"] == 1   # each one-wave workgroup's own rows
        assert_update_parity(dev, orc, "32768x64 upd %d" % j, stats=stats)
    print("cost errors (rel, /Delta, (J-Jmin)/Delta):", stats)


def _hip():
    L = C.CDLL("libamdhip64.so.7")
    L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    L.hipDeviceSynchronize.argtypes = []
    return L


@pytest.mark.parametrize("S,horison,window", [(32768, 0.64, 0), (65536, 1.28, 10)])
def test_eight_shards_equal_unsharded(S, horison, window):
    """configs[3]'s and configs[4]'s partition on one GPU: eight phase-split handles
    (the reference's ThreadPool split, mppi.cpp:277-302: 4096 or 4097 rollouts each for configs[3];
    8192 or 8193 for configs[4], whose first two ranks run the two-launch split and the rest one
    round of one-wave workgroups), with the two all-reduces done on the host between the phases,
    against one handle of all S + 2 rollouts (device Philox: draws are keyed by global rollout, so
    every rank draws what the single handle draws).  configs[4] with the Savitzky-Golay filter."""
    sg = am.Smoothing(window, 1) if window else None
    conf = am.frankaridgeback_configuration(rollouts=S, horison=horison, keep_best_rollouts=20, threads=8, smoothing=sg)
    mk = lambda: am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    world = 8
    single, shards = mk(), [mk() for _ in range(world)]
    for r, t in enumerate([single] + shards):
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        if t is not single:
            t.set_shard(world, r - 1)
    hip = _hip()
    R, HC = single.R, single.H * single.C
    x = am.huddled_state()
    loose = 1.0 if single.H <= 64 else 10.0
    worst = (0.0, 0.0, 0.0)

    def allreduce(ptrs, n):
        bufs = [np.zeros(n) for _ in ptrs]
        for p, b in zip(ptrs, bufs):
            assert hip.hipMemcpy(b.ctypes.data, p, n * 8, 2) == 0   # D2H
        s = bufs[0].copy()
        for b in bufs[1:]:
            s += b
        for p in ptrs:
            assert hip.hipMemcpy(p, s.ctypes.data, n * 8, 1) == 0   # H2D

    for j in range(3):
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
        for r, sh in enumerate(shards):
            b, e = am.shard_range(R, world, r)
            mine, ref = sh.noise()[b:e], full[b:e]
            d = max(2 - b, 0)   # rollout 1 carries -U*, which differs in the last bits (gradient order)
            np.testing.assert_array_equal(mine[d:], ref[d:], err_msg="update %d shard %d noise" % (j, r))
            np.testing.assert_allclose(mine[:d], ref[:d], rtol=0, atol=1e-12)
            if j > 0 and (e - b) % 8192 != 0:   # rounds of four-wave groups (or the split): draws ahead
                assert sh.update_info()["sampling"] == 2
        for sh in shards:
            # update 0 starts from U* = 0 on both sides: identical bits.  After it, U* carries the
            # last bits of the gradient's summation order (eight partial sums all-reduced against
            # one), and every rollout rolls out U*_shifted + eps: measured up to 4.3e-12 relative
            # (rollout 31767, update 2), so the Delta bar of assert_update_parity
            # H = 128 compounds the last bits over twice the steps (as in the oracle parity at H = 128)
            cs, cu = sh.costs(), single.costs()
            if j == 0:
                np.testing.assert_array_equal(cs, cu)
            delta = np.nanmax(cu) - np.nanmin(cu)
            bar = loose * 1e-11 * (delta + np.abs(cu))
            bad = np.abs(cs - cu) > bar
            assert not bad.any(), "rollout %d: %r vs %r" % (int(np.argmax(bad)), cs[np.argmax(bad)], cu[np.argmax(bad)])
            du = np.max(np.abs(sh.get_optimal_rollout() - single.get_optimal_rollout()))
            dw = np.max(np.abs(sh.get_weights() - single.get_weights()))
            worst = tuple(max(w, v) for w, v in zip(worst, (np.nanmax(np.abs(cs - cu)) / delta, du, dw)))
            # weights: 1.1e-14 measured at 65536 x 128 SG (r06, the Gauss-Jordan with one row per
            # lane), 4.1e-15 before it: the bar is 3e-15 per unit of loose
            assert du <= loose * 1e-12 and dw <= loose * 3e-15, (du, dw)
            assert sh.argmin() == single.argmin()
    print("worst (cost error / Delta, U* abs, weights abs):", worst)


@pytest.mark.parametrize("S,updates", [(8192, 3), (65536, 2)])
def test_config4_savitzky_golay_h128(S, updates):
    """configs[4]: H = 128 with the Savitzky-Golay filter (window 10, order 1) fused into the
    finish launch (sg_finish_kernel); 8192 is its per-GPU share at N = 8, 65536 its total."""
    conf, dev, orc, sd = fr_pair(S=S, horison=1.28, smoothing=am.Smoothing(10, 1), threads=THREADS)
    rng = np.random.default_rng(S)
    x = am.huddled_state()
    stats = []
    for j in range(updates):
        step_both(dev, orc, x, 0.05 * j, rng, sd)
        # H = 128: the two solves' last-bit differences compound over twice the steps (measured
        # 1.67e-11 and 3.33e-11 of Delta, 1.02e-11 relative, at 65536 x 128): both bars are 1e-10
        # here, still five orders inside the fp32-class tolerance north_star asks for
        assert_update_parity(dev, orc, "%dx128 SG upd %d" % (S, j), stats=stats, cost_dfrac=1e-10, cost_rtol=1e-10)
    uu_d, tt_d, st_d = dev.smoothing_windows()
    uu_o, tt_o, st_o = orc.smoothing_windows(10)
    np.testing.assert_array_equal(tt_d, tt_o)
    np.testing.assert_array_equal(st_d, st_o)
    np.testing.assert_allclose(uu_d, uu_o, rtol=0, atol=1e-9)
    print("cost errors (rel, /Delta, (J-Jmin)/Delta):", stats)


@pytest.mark.parametrize("rollouts,horison,window", [(4096, 0.64, 0), (1000, 0.64, 0), (4096, 1.28, 10), (8192, 1.28, 10),
                                                     (4094, 0.64, 0), (8200, 0.32, 0)])
def test_graph_path_equals_eager_launches(rollouts, horison, window):
    """The hipGraph path of update() (mppi_set_graph: the steady-state update captured once and
    replayed with each update's arguments written into its kernel nodes) gives the eager launches'
    bits over updates with varying shifts (5, 2, 5, 0 steps), including a state change and an
    interruption (reading the optimal cost runs filter() by itself, so the next update is eager).
    4096 x 128 with the Savitzky-Golay filter (window 10): configs[4]'s filter, sg_finish_kernel as
    the graph's finish node; 8192 x 128 with it is configs[4]'s share per GPU, whose rollouts are
    the two-launch split (five kernel nodes).  4094 rollouts (R = 4096, a multiple of 16 rows)
    leave filter() pending in a four-wave launch, a shape the graph does not replay: every update
    runs eagerly (such a handle once failed every other update).  8200 rollouts rank
    past RANK_TILED_MAX: the chunk + merge rank launches replay with their captured arguments."""
    sg = am.Smoothing(window, 1) if window else None
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8,
                                            smoothing=sg)
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22, 0.27, 0.32]
    out = {}
    for graph in (0, 1):
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.set_graph(graph)
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for j, tm in enumerate(times):
            if j == 5:
                x = x.copy()
                x[12 + 4] = 0.3
            t.update(x, tm)
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
            if j == 6:
                rec.append(t.get_optimal_total_cost())
        out[graph] = (rec, t.graph_updates())
    graphable = (rollouts + 2) % 16 != 0
    assert out[0][1] == 0 and (out[1][1] >= 5 if graphable else out[1][1] == 0), out[1][1]
    for j, (a, b) in enumerate(zip(out[0][0], out[1][0])):
        if isinstance(a, float):
            assert a == b
            continue
        for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))


def test_c_update_entry_equals_update():
    """bench.py's timed loop (the C-ABI mppi_update called directly through c_update_entry) against
    Trajectory.update on a twin handle: the same costs, gradient, U* and optimal cost, bit for bit,
    over five updates of the bench workload."""
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.64, keep_best_rollouts=20, threads=THREADS)
    a = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    b = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    x = am.huddled_state()
    for t in (a, b):
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
    fn, h, ptr = b.c_update_entry(x)
    for j in range(5):   # (one handle's launches at a time: each launch wants every CU)
        a.update(x, 0.05 * j)
        a.synchronize()
        assert fn(h, ptr, 0.05 * j) == abi.MPPI_OK
        b.synchronize()
    np.testing.assert_array_equal(a.costs(), b.costs())
    np.testing.assert_array_equal(a.get_gradient(), b.get_gradient())
    np.testing.assert_array_equal(a.get_optimal_rollout(), b.get_optimal_rollout())
    assert a.get_optimal_total_cost() == b.get_optimal_total_cost()
    np.testing.assert_array_equal(b.state_buffer, x)
    a.close()
    b.close()
