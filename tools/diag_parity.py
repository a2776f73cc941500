"""Per-rollout device-vs-oracle cost comparison for one FrankaRidgeback update (GPU box)."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import assistedmanipulation_amd as am  # noqa: E402
from helpers import fr_pair, step_both  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
H = float(sys.argv[2]) if len(sys.argv) > 2 else 0.32
conf, dev, orc, sd = fr_pair(S=S, horison=H)
rng = np.random.default_rng(12345)
step_both(dev, orc, am.huddled_state(), 0.0, rng, sd)
cd, co = dev.costs(), orc.costs()
rel = np.abs(cd - co) / np.maximum(np.abs(co), 1.0)
print("rel err: max %.3e median %.3e; >1e-9: %d of %d" % (np.nanmax(rel), np.nanmedian(rel), int(np.sum(rel > 1e-9)), len(rel)))
bad = np.argsort(-np.nan_to_num(rel))[:8]
for i in bad:
    print("  rollout %4d dev %.17g oracle %.17g rel %.3e" % (i, cd[i], co[i], rel[i]))
print("costs[0:4] dev", cd[:4], "oracle", co[:4])
