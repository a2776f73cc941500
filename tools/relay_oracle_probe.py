"""Which side is right when the relay in one workgroup (MPPI_RELAY_K=1) and over two (K=2) disagree
(a GPU diagnostic): the relay_race_probe sequence with the device's draws replayed through the oracle
(tests/helpers.py replay_device_draws); per update, each handle's worst cost error against the oracle
relative to the cost spread, and the rollouts past 1e-9 of it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import assistedmanipulation_amd as am  # noqa: E402
from assistedmanipulation_amd import abi  # noqa: E402
from oracle import oracle as O  # noqa: E402
from helpers import replay_device_draws  # noqa: E402


def main(rollouts=1000, horison=0.64):
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22, 0.27]
    for k in (1, 2):
        os.environ["MPPI_RELAY_K"] = str(k)
        conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8)
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
        for j, t in enumerate(times):
            if j == 5:
                x = x.copy()
                x[12 + 4] = 0.3
            costs, noise = replay_device_draws(dev, orc, x, t, prev_costs, prev_noise, 20)
            co = orc.costs()
            ok = np.isfinite(co)
            delta = np.nanmax(co) - np.nanmin(co)
            err = np.abs(costs - co) / delta
            bad = np.flatnonzero(err > 1e-9)
            print("K=%d update %d: worst err/Delta %.3e, rollouts past 1e-9: %s" % (k, j, np.nanmax(err[ok]), bad.tolist()[:10]),
                  flush=True)
            prev_costs, prev_noise = costs, noise
            # the oracle follows the device's U* only through the same costs: stop at the first divergence
            if len(bad):
                break


if __name__ == "__main__":
    main()
