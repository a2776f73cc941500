"""Effective shader clock of each dispatch: GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / wall
time (MI355X_MICROARCH.md, DVFS give-back).  usage: clock_probe.py <dir> <prefix>"""
import collections
import csv
import os
import sys

d, pre = sys.argv[1], sys.argv[2]
cnt = {}
for r in csv.DictReader(open(os.path.join(d, pre + "_counter_collection.csv"))):
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
        cnt[r["Dispatch_Id"]] = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]), float(r["Counter_Value"]))
dur = {}
trace = os.path.join(d, pre + "_kernel_trace.csv")
if os.path.exists(trace):
    for r in csv.DictReader(open(trace)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(list)
for k, (name, grid, g) in cnt.items():
    if k in dur and dur[k] > 0:
        agg[(name, grid)].append((g / 8 / dur[k] / 1e9, dur[k] * 1e3))
for (name, grid), v in sorted(agg.items()):
    if "coop" in name:
        print("%-40s grid %7d  clock %.2f GHz  dur %.3f ms  (n=%d)" % (name[:40], grid, sum(x[0] for x in v) / len(v),
                                                                   sum(x[1] for x in v) / len(v), len(v)))
