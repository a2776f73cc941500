"""The sharded update path through RCCL on one GPU.

One process per GPU is the multi-GPU layout, and the round's GPU box has one GPU, so RCCL cannot
form a two-rank communicator here (two ranks on one device are refused as duplicate GPUs).  A
one-rank communicator (mppi_comm_init with world 1) still runs the sharded path end to end:
ncclCommInitRank, the rollout launch writing the local cost vector, ncclAllReduce of the costs on
the engine stream, the weights from a pass over the all-reduced costs (not the rollout launch's
cost statistics), ncclAllReduce of the partial gradient, then the publish.  It must equal the unsharded handle: the noise and the costs bit for
bit, U* to the gradient's summation order (mppi.cpp:344-448).

The sharded update as a captured hipGraph (configs[4]: "8 x MI355X ... hipGraph-captured control
step"): the rollout launch(es), ncclAllReduce of the costs, the weight reduce, ncclAllReduce of the
partial gradient, the finish and the rank + next draws captured once, RCCL's nodes included, and
replayed with each update's arguments: bit-identical to the eager sharded launches.
"""
import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rollouts,horison", [(1000, 0.32), (4096, 0.64)])
def test_one_rank_rccl_equals_unsharded(rollouts, horison):
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8)
    mk = lambda: am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    plain, rccl = mk(), mk()
    rccl.comm_init(1, 0, am.comm_unique_id())
    info = rccl.comm_info()   # what RCCL reports (ncclCommCount / ncclCommUserRank), and the device
    assert info["nranks"] == 1 and info["rank"] == 0 and info["pci_bus_id"], info
    assert plain.comm_info()["nranks"] == 0 and plain.comm_info()["pci_bus_id"] == info["pci_bus_id"]
    for t in (plain, rccl):
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
    x = am.huddled_state()
    for j, tm in enumerate([0.0, 0.05, 0.07, 0.12, 0.17]):
        plain.update(x, tm)
        rccl.update(x, tm)
        cp, cr = plain.costs(), rccl.costs()
        # rollout 1 carries -U*, whose last bits follow the gradient's summation order
        np.testing.assert_array_equal(rccl.noise()[2:], plain.noise()[2:], err_msg="update %d noise" % j)
        np.testing.assert_allclose(rccl.noise()[:2], plain.noise()[:2], rtol=0, atol=1e-12)
        if j == 0:
            np.testing.assert_array_equal(cr, cp, err_msg="update 0 costs")
        else:
            finite = np.isfinite(cp)
            delta = cp[finite].max() - cp[finite].min()
            assert np.array_equal(np.isfinite(cr), finite)
            assert np.max(np.abs(cr[finite] - cp[finite])) <= 1e-11 * delta, "update %d costs" % j
        assert rccl.argmin() == plain.argmin()
        np.testing.assert_allclose(rccl.get_weights(), plain.get_weights(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(rccl.get_optimal_rollout(), plain.get_optimal_rollout(), rtol=0, atol=1e-12)


@pytest.mark.parametrize("rollouts,horison,window", [(4096, 0.64, 0), (8192, 1.28, 10), (8200, 0.32, 0)])
def test_sharded_graph_equals_eager(rollouts, horison, window):
    """Through a one-rank communicator: the graph path (mppi_set_graph) against the eager sharded
    launches, over updates with varying shifts (5, 2, 5, 0 steps), a state change and an
    interruption (reading the optimal cost runs filter() by itself; the next update is eager).
    8192 x 128 with the Savitzky-Golay filter is configs[4]'s share per GPU (the two-launch split,
    sg_finish_kernel); 8200 rollouts rank past RANK_TILED_MAX (the chunk + merge rank launches stay
    in the graph with their captured arguments)."""
    sg = am.Smoothing(window, 1) if window else None
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8,
                                            smoothing=sg)
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22, 0.27, 0.32]
    out = {}
    for graph in (0, 1):
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.comm_init(1, 0, am.comm_unique_id())
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
    assert out[0][1] == 0 and out[1][1] >= 5, out[1][1]
    for j, (a, b) in enumerate(zip(out[0][0], out[1][0])):
        if isinstance(a, float):
            assert a == b
            continue
        for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))


@pytest.mark.parametrize("rollouts,horison", [(4096, 0.64)])
def test_graph_capture_failure_runs_the_update_eagerly(rollouts, horison):
    """a capture that fails after the update (its RCCL all-reduces included) was
    recorded - here an injected instantiation failure (MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL) - must
    still run that update, eagerly and with its two collectives, from the host state it started
    from, so that peer ranks replaying the graph are not left blocked in an all-reduce; the handle
    stays eager.  Bit-identical to a handle that never tried the graph."""
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8)
    times = [0.0, 0.05, 0.07, 0.12, 0.17]
    out = {}
    for graph in (0, 1):
        t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
        t.comm_init(1, 0, am.comm_unique_id())
        t.set_graph(graph)
        if graph:
            t.debug_inject(abi.MPPI_DEBUG_GRAPH_INSTANTIATE_FAIL, 1)
        t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
        t.set_forecast(am.constant_forecast(t.H))
        x = am.huddled_state()
        rec = []
        for tm in times:
            t.update(x, tm)
            rec.append((t.noise().copy(), t.costs().copy(), t.get_optimal_rollout().copy(), t.get_weights().copy()))
        out[graph] = (rec, t.update_info())
    info = out[1][1]
    assert info["graph_failures"] == 1 and info["graph_updates"] == 0, info
    assert info["update_count"] == len(times) == out[0][1]["update_count"]
    for j, (a, b) in enumerate(zip(out[0][0], out[1][0])):
        for name, u, v in zip(("noise", "costs", "optimal", "weights"), a, b):
            np.testing.assert_array_equal(u, v, err_msg="update %d %s" % (j, name))
