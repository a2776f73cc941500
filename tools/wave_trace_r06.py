"""COOP_TRACE + COST_TRACE wave trace of the 4096 x 64 update launch (MPPI_WAVE_TRACE): where the
launch's end comes from.  Per main wave (slot 4 w + ...): [0] loop start, [1] loop end, [2] HW_ID,
[3] the wave's end after its objective work; slot 1024: the relay's start / end, 1025: the relay
stages' ends; 1040 + 4 g + c: block 0's cost chunk c of group g (start, end, wave).
usage: wave_trace_r06.py file [nslots=1064]"""
import sys

import numpy as np

path = sys.argv[1]
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 1064
raw = np.fromfile(path, dtype=np.uint32)
recs = raw.reshape(-1, ns, 4).astype(np.int64)
nmain = 1024
q = lambda a: "min %6.1f p10 %6.1f p50 %6.1f p90 %6.1f max %6.1f" % (a.min(), np.percentile(a, 10), np.median(a),
                                                                  np.percentile(a, 90), a.max())
for u in (len(recs) // 2, len(recs) - 1):
    rec = recs[u]
    st, le, hw, we = rec[:nmain, 0], rec[:nmain, 1], rec[:nmain, 2], rec[:nmain, 3]
    t0 = st[st > 0].min()
    us = lambda x: (x - t0) / 100.0
    print("update %d of %d" % (u, len(recs)))
    print("  main loop start :", q(us(st)))
    print("  main loop end   :", q(us(le)))
    print("  main wave end   :", q(us(we)))
    print("  tail (end - loop end):", q((we - le) / 100.0))
    blk = np.arange(nmain) // 4
    bend = np.array([us(we[blk == b]).max() for b in range(256)])
    bloop = np.array([us(le[blk == b]).max() for b in range(256)])
    print("  workgroup end   :", q(bend))
    order = np.argsort(-bend)[:8]
    print("  last workgroups :", ", ".join("b%d %.1f (loops %.1f)" % (b, bend[b], bloop[b]) for b in order))
    # per-XCD (blocks round-robin over 8 XCDs)
    print("  per XCD end p50 :", " ".join("%.1f" % np.median(bend[x::8]) for x in range(8)))
    fx = rec[nmain]
    print("  relay rows: start %.1f end %.1f, stages end" % (us(fx[0]), us(fx[1])),
          ["%.1f" % us(x) for x in rec[nmain + 1]])
    for m in range(1, 4):   # members 1..3 of a relay over several workgroups (MPPI_RELAY_K)
        if rec[nmain + 1 + m].any():
            print("  relay member %d stages end" % m, ["%.1f" % us(x) if x else "-" for x in rec[nmain + 1 + m]])
    for g in range(5):
        row = []
        for c in range(4):
            s0, s1, wv, _ = rec[nmain + 16 + 4 * g + c]
            row.append("%.1f-%.1f w%d" % (us(s0), us(s1), wv) if s0 else "-")
        print("  block 0 group %d chunks:" % g, "  ".join(row))
