"""COOP_TRACE + COST_TRACE builds (MPPI_WAVE_TRACE): per main wave the horizon loop's start and end
and the wave's end after its objective rows; the fifth wave's slot holds its loop start and the
end of its rows (by the fifth wave or, after take_over, by the wave that took them).
usage: wave_trace_r03.py file nslots"""
import sys

import numpy as np

path, ns = sys.argv[1], int(sys.argv[2])
raw = np.fromfile(path, dtype=np.uint32)
rec = raw.reshape(-1, ns, 4)[-1].astype(np.int64)
nmain = 1024
st, le, we = rec[:nmain, 0], rec[:nmain, 1], rec[:nmain, 3]
t0 = st[st > 0].min()
us = lambda x: (x - t0) / 100.0
q = lambda a: "min %.1f p50 %.1f p90 %.1f max %.1f" % (a.min(), np.median(a), np.percentile(a, 90), a.max())
print("main loop start  us:", q(us(st)))
print("main loop end    us:", q(us(le)))
print("main wave end    us:", q(us(we)))
print("block 0 waves: loop end", ["%.1f" % us(le[w]) for w in range(4)], "wave end", ["%.1f" % us(we[w]) for w in range(4)])
fx = rec[nmain]
print("fifth wave rows: start %.1f end %.1f" % (us(fx[0]), us(fx[1])))
print("launch end (last wave end) %.1f us" % max(us(we).max(), us(fx[1])))
if len(sys.argv) > 3 and sys.argv[3] == "relay":   # relay builds: block 0's stage ends in the next slot
    print("relay stage ends:", ["%.1f" % us(x) for x in rec[nmain + 1]])
if len(sys.argv) > 3 and ns >= 1024 + 16 + 20:   # COST_TRACE builds: block 0's chunks (start, end, wave), group-major
    for g in range(5):
        row = []
        for c in range(4):
            s0, s1, wv, _ = rec[nmain + 16 + 4 * g + c]
            row.append("%.1f-%.1f w%d" % (us(s0), us(s1), wv) if s0 else "-")
        print("block 0 group %d chunks:" % g, "  ".join(row))
