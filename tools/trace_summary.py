"""Average kernel durations (us) from a rocprofv3 kernel_trace.csv; the rollout kernel's main
and single-rollout (filter) dispatches are listed separately."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    if "rollout" in n or "coop" in n:
        n += "[main]" if g > 64 else "[single]"
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for n, v in sorted(d.items(), key=lambda x: -sum(x[1]) / len(x[1])):
    print("%-44s n=%3d avg=%9.1f us" % (n[:44], len(v), sum(v) / len(v)))
