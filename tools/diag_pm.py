"""Diagnose point-mass parity: which rollouts / noise columns differ after update 0."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from helpers import pm_pair, step_both

conf, dev, orc, sd = pm_pair(S=1024, horison=0.32)
rng = np.random.default_rng(12345)
x = np.zeros(6)
step_both(dev, orc, x, 0.0, rng, sd)
cd, co = dev.costs(), orc.costs()
bad = np.nonzero(np.abs(cd - co) > 1e-9 * np.maximum(1, np.abs(co)))[0]
print("bad rollouts", len(bad), bad[:40])
nd, no = dev.noise(), orc.noise()
print("noise shape", nd.shape)
nb = np.nonzero(np.any(np.abs(nd - no) > 0, axis=(1, 2)))[0]
print("noise-diff rollouts", len(nb), nb[:40])
print("weights diff", np.max(np.abs(dev.get_weights() - orc.weights())))
