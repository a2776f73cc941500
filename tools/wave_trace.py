"""Analyse MPPI_WAVE_TRACE output (COOP_TRACE builds): per-block start/end (100 MHz realtime),
hardware placement (XCC, SE, CU, SIMD), co-residency.  usage: wave_trace.py file nblocks"""
import collections
import sys

import numpy as np

path, nb = sys.argv[1], int(sys.argv[2])
raw = np.fromfile(path, dtype=np.uint32)
rec = raw.reshape(-1, nb, 4)[-1].astype(np.int64)   # last update
rec = rec[:nb]
st, en, hw, xcc = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3] & 0xF
ok = en != 0
st, en, hw, xcc = st[ok], en[ok], hw[ok], xcc[ok]
t0 = st.min()
s_us, e_us = (st - t0) / 100.0, (en - t0) / 100.0   # 100 MHz -> us
dur = e_us - s_us
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = list(zip(xcc, se, sh, cu, simd))
cnt = collections.Counter(key)
cu_cnt = collections.Counter(zip(xcc, se, sh, cu))
print("blocks %d  distinct SIMDs %d  distinct CUs %d" % (len(st), len(cnt), len(cu_cnt)))
print("waves per SIMD histogram:", sorted(collections.Counter(cnt.values()).items()))
print("waves per CU histogram:", sorted(collections.Counter(cu_cnt.values()).items()))
print("start  us: min %.1f  p50 %.1f  p90 %.1f  max %.1f" % (s_us.min(), np.median(s_us), np.percentile(s_us, 90), s_us.max()))
print("end    us: min %.1f  p50 %.1f  p90 %.1f  max %.1f" % (e_us.min(), np.median(e_us), np.percentile(e_us, 90), e_us.max()))
print("dur    us: min %.1f  p50 %.1f  p90 %.1f  max %.1f" % (dur.min(), np.median(dur), np.percentile(dur, 90), dur.max()))
share = np.array([cnt[k] for k in key])
cus = np.array([cu_cnt[(a, b, c, d)] for a, b, c, d, _ in key])
for n in sorted(set(cus)):
    m = cus == n
    print("  blocks on CUs holding %d waves: %4d  dur p50 %.1f us" % (n, m.sum(), np.median(dur[m])))
for n in sorted(set(share)):
    m = share == n
    print("  blocks on SIMDs holding %d waves: %4d  dur p50 %.1f us" % (n, m.sum(), np.median(dur[m])))
print("per-XCC blocks:", sorted(collections.Counter(xcc).items()))
order = np.argsort(-dur)[:6]
idx = np.nonzero(ok)[0]
for i in order:
    print("  longest: wave %5d dur %.1f us start %.1f end %.1f  SIMD %s (waves there %d)" % (idx[i], dur[i], s_us[i], e_us[i], key[i], cnt[key[i]]))
