"""Quick per-library check on the GPU (A/B builds via MPPI_AMD_LIB): a few updates at 128 and 4096
rollouts with the fifth wave's rows handed over or not; prints the update info (handover step, wait
timeouts) and a digest of the costs, weights and U*, so builds can be compared bit for bit."""
import hashlib
import os
import sys
import time

import numpy as np

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi


def digest(*arrs):
    h = hashlib.sha1()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:12]


def main():
    for S in (128, 4096):
        for ho in ("0", "1"):
            os.environ["MPPI_HANDOVER"] = ho
            conf = am.frankaridgeback_configuration(rollouts=S, horison=0.64, keep_best_rollouts=20, threads=8)
            t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
            t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
            t.set_forecast(am.constant_forecast(t.H))
            x = am.huddled_state()
            t0 = time.time()
            for j in range(4):
                t.update(x, 0.05 * j)
            t.synchronize()
            dt = (time.time() - t0) / 4
            info = t.update_info()
            c = t.costs()
            print("S=%d ho=%s %.3f ms/update info=%s costs[min,max]=(%.6e, %.6e) digest=%s" % (
                S, ho, dt * 1e3, {k: info[k] for k in ("handover", "wait_timeouts", "rows")}, np.nanmin(c), np.nanmax(c),
                digest(c, t.get_weights(), t.get_optimal_rollout())), flush=True)


if __name__ == "__main__":
    main()
