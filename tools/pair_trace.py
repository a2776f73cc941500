import numpy as np, sys
raw = np.fromfile(sys.argv[1], dtype=np.uint32)
ns = 1064
rec = raw.reshape(-1, ns, 4).astype(np.int64)
for u in (-1, -2, -3):
    r = rec[u]
    st, le, we = r[:1024, 0], r[:1024, 1], r[:1024, 3]
    t0 = st[st > 0].min()
    us = lambda x: (np.asarray(x) - t0) / 100.0
    print("update", u)
    print("  block 0 stage ends", np.round(us(r[1025]), 1), " block 8 stage ends", np.round(us(r[1033]), 1))
    print("  token at stage 4 %.1f, first-half sums %.1f, second-half J %.1f" % (us(r[1063][2]), us(r[1063][1]), us(r[1063][0])))
    for b in (0, 8):
        print("  block %d main loop ends" % b, np.round(us(le[4*b:4*b+4]), 1), "wave ends", np.round(us(we[4*b:4*b+4]), 1))
    bw = us(we).reshape(256, 4).max(1)
    print("  wave end: p50 %.1f, max excl 0/8 %.1f, block 8 %.1f" % (np.median(bw), np.delete(bw, [0, 8]).max(), bw[8]))
