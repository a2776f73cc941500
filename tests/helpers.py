"""Shared setup for the parity tests: paired device / oracle trajectories driven with the same
injected noise stream (Gaussian eps with the configured variances, seeded)."""
import numpy as np

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi
from oracle import oracle as O

# fp64 on both sides, different operation order (world-frame zero-bias ABA with FMA contraction
# on the device vs Pinocchio-order RNEA + ABA without contraction in the oracle): observed
# relative differences are ~1e-15; the bounds below leave two to three orders of margin.
COST_RTOL = 1e-11        # per-rollout cost, relative to |cost|
WEIGHT_ATOL = 1e-11
CONTROL_ATOL = 1e-9      # U*, gradient (controls reach O(100) for arm torques)


def energy_only_cost():
    """AssistedManipulation with only enable_energy_limit set (gen_golden.energy_only_cost): the
    rollout cost is then the tank's barrier alone, so the parity bars measure the energy path."""
    cost = am.AssistedManipulation()
    c = cost.configuration
    c.enable_joint_limit = c.enable_self_collision_limit = c.enable_workspace_limit = 0
    c.enable_velocity_cost = c.enable_trajectory_cost = c.enable_manipulability_cost = 0
    c.enable_energy_limit = 1
    return cost


def fr_pair(S, horison, K=20, smoothing=None, mode=0, threads=8, forecast=True, cost=None):
    conf = am.frankaridgeback_configuration(rollouts=S, horison=horison, keep_best_rollouts=K,
                                            smoothing=smoothing, threads=threads)
    dyn = am.FrankaRidgebackDynamics()
    cost = cost if cost is not None else am.AssistedManipulation()
    dev = am.Trajectory.create(conf, dyn, cost)
    assert dev is not None
    dev.set_noise_source(abi.MPPI_NOISE_HOST_INJECTED)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dyn.descriptor(), cost.descriptor(), scalar=0, mode=mode)
    if forecast:
        table = am.constant_forecast(dev.H)
        dev.set_forecast(table)
        orc.set_forecast(table)
    return conf, dev, orc, np.sqrt(np.diag(conf.covariance))


def pm_pair(S=1024, horison=0.32, K=20):
    conf = am.point_mass_configuration(rollouts=S, horison=horison, keep_best_rollouts=K)
    dyn, cost = am.PointMassDynamics(), am.QuadraticCost()
    dev = am.Trajectory.create(conf, dyn, cost)
    assert dev is not None
    dev.set_noise_source(abi.MPPI_NOISE_HOST_INJECTED)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dyn.descriptor(), cost.descriptor())
    return conf, dev, orc, np.sqrt(np.diag(conf.covariance))


def step_both(dev, orc, state, time, rng, sd):
    n = orc.noise_draws(time)
    assert dev.noise_draws(time) == n
    eps = rng.standard_normal((n, len(sd))) * sd
    dev.inject_noise(eps)
    orc.inject_noise(eps)
    orc.update(state, time)
    dev.update(state, time)


def assert_update_parity(dev, orc, tag="", cost_rtol=COST_RTOL, weight_atol=WEIGHT_ATOL):
    cd, co = dev.costs(), orc.costs()
    assert np.array_equal(np.isnan(cd), np.isnan(co)), tag + " NaN pattern differs"
    ok = ~np.isnan(co)
    rel = np.abs(cd[ok] - co[ok]) / np.maximum(np.abs(co[ok]), 1.0)
    assert rel.max() <= cost_rtol, "%s cost rel err %.3e at %d" % (tag, rel.max(), int(np.argmax(rel)))
    assert int(np.nanargmin(cd)) == int(np.nanargmin(co)), tag + " argmin differs"
    assert dev.argmin() == int(np.nanargmin(co))
    np.testing.assert_allclose(dev.get_weights(), orc.weights(), rtol=0, atol=weight_atol, err_msg=tag + " weights")
    np.testing.assert_allclose(dev.get_gradient(), orc.gradient(), rtol=0, atol=CONTROL_ATOL, err_msg=tag + " gradient")
    np.testing.assert_allclose(dev.get_optimal_rollout(), orc.optimal_control(), rtol=0, atol=CONTROL_ATOL,
                               err_msg=tag + " U*")
    od, oo = dev.get_optimal_total_cost(), orc.optimal_cost()
    assert abs(od - oo) <= cost_rtol * max(abs(oo), 1.0), "%s optimal cost %r vs %r" % (tag, od, oo)
    return rel.max()
