"""The sharded update path through RCCL on one GPU.

One process per GPU is the multi-GPU layout, and the round's GPU box has one GPU, so RCCL cannot
form a two-rank communicator here (two ranks on one device are refused as duplicate GPUs).  A
one-rank communicator (mppi_comm_init with world 1) still runs the sharded path end to end:
ncclCommInitRank, the rollout launch writing the local cost vector, ncclAllReduce of the costs on
the engine stream, the weights from a pass over the all-reduced costs (not the rollout launch's
cost statistics), ncclAllReduce of the partial gradient, then the publish.  It must equal the unsharded handle: the noise and the costs bit for
bit, U* to the gradient's summation order (mppi.cpp:344-448).
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
