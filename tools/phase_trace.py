"""Per-phase shader cycles of the rollout kernel's step (PHASE_TRACE builds, MPPI_WAVE_TRACE file):
mean over the main waves of the last update.  usage: phase_trace.py file nwaves"""
import sys

import numpy as np

path, nw = sys.argv[1], int(sys.argv[2])
fk = len(sys.argv) > 3 and sys.argv[3] == "fk"
raw = np.fromfile(path, dtype=np.uint32)
rec = raw.reshape(-1, nw, 4)[-1].astype(np.float64)[:1024]
rec = rec[rec.sum(axis=1) > 0]
names = ["FK+record", "ABA backward", "ABA forward", "integrate+sincos"]
if fk:
    names = ["FK pre-scan", "FK scan", "inertia+S+LDS", "EE+kin sums"]
tot = rec.sum(axis=1).mean()
for i, n in enumerate(names):
    print("%-18s %8.0f cycles/step  %5.1f %%" % (n, rec[:, i].mean() / 63.0, 100.0 * rec[:, i].mean() / tot))
print("%-18s %8.0f cycles/step (%d waves)" % ("total", tot / 63.0, len(rec)))
