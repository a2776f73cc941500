"""Diagnostics: per-rollout cost mismatch device vs oracle on one small FrankaRidgeback update
(run on the GPU box; MPPI_AMD_LIB selects a variant).  usage: diag_costs.py [S] [horizon_s]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from helpers import fr_pair, step_both  # noqa: E402
import assistedmanipulation_amd as am  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hor = float(sys.argv[2]) if len(sys.argv) > 2 else 0.32
conf, dev, orc, sd = fr_pair(S=S, horison=hor)
rng = np.random.default_rng(12345)
x = am.huddled_state()
for j in range(2):
    step_both(dev, orc, x, 0.05 * j, rng, sd)
    cd, co = dev.costs(), orc.costs()
    rel = np.abs(cd - co) / np.maximum(np.abs(co), 1.0)
    bad = np.nonzero(rel > 1e-11)[0]
    print("update %d: %d of %d rollouts off; max rel %.3e" % (j, len(bad), len(cd), np.nanmax(rel)))
    print("  bad rollouts:", bad[:40].tolist())
    print("  bad rollouts mod 16:", sorted(set((bad % 16).tolist())), " row-in-wave (r//4 %% 4):", sorted(set(((bad // 4) % 4).tolist())))
