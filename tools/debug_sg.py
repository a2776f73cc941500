"""Debug: per-update SG window comparison device vs oracle (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import assistedmanipulation_amd as am
from helpers import fr_pair, step_both
conf, dev, orc, sd = fr_pair(S=128, horison=0.64, smoothing=am.Smoothing(10, 1))
rng = np.random.default_rng(3)
x = am.huddled_state()
for j in range(5):
    step_both(dev, orc, x, 0.05 * j, rng, sd)
    ud, td, sdv = dev.smoothing_windows()
    uo, to, so = orc.smoothing_windows(10)
    print(j, "start", sdv[:3], so[:3], "tt eq", np.array_equal(td, to), "uu maxdiff", np.abs(ud - uo).max(),
          "U* diff", np.abs(dev.get_optimal_rollout() - orc.optimal_control()).max())
    if not np.array_equal(td, to):
        bad = np.argwhere(td != to)
        print("  tt diffs at", bad[:5], td[bad[0][0], bad[0][1]], to[bad[0][0], bad[0][1]])
        print("  td row0", td[0, :20]); print("  to row0", to[0, :20])
    d = np.abs(ud - uo)[0]
    print("  uu row0 diff idx", np.nonzero(d > 1e-12)[0][:20])
