"""Per-kernel averages of a rocprofv3 counter-collection CSV; the rollout kernel's main
(multi-wave) dispatches are separated from its single-rollout (filter) dispatches."""
import collections
import csv
import sys


def summarize(path):
    rows = list(csv.DictReader(open(path)))
    disp = collections.defaultdict(dict)
    for r in rows:
        name = r["Kernel_Name"]
        name = name[:name.rfind("(")] if name.endswith(")") else name   # drop the argument list
        key = (r["Dispatch_Id"], name.replace("(anonymous namespace)::", ""))
        disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
        disp[key]["_grid"] = int(r["Grid_Size"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (d, name), c in disp.items():
        tag = name + ("[main]" if c["_grid"] > 64 else "[single]") if "rollout" in name or "coop" in name else name
        for k, v in c.items():
            agg[tag][k].append(v)
    out = {}
    for tag, c in agg.items():
        out[tag] = {k: sum(v) / len(v) for k, v in c.items()}
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    for tag, c in sorted(res.items()):
        line = " ".join("%s=%.4g" % (k, v) for k, v in sorted(c.items()))
        if "SQ_WAVES" in c and c["SQ_WAVES"] > 0 and "SQ_INSTS_VALU" in c:
            w = c["SQ_WAVES"]
            line += " | per-wave: valu=%.0f lds=%.0f wave_cyc=%.0f active=%.2f wait=%.2f" % (
                c["SQ_INSTS_VALU"] / w, c.get("SQ_INSTS_LDS", 0) / w, c.get("SQ_WAVE_CYCLES", 0) / w,
                c.get("SQ_ACTIVE_INST_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)),
                c.get("SQ_WAIT_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)))
        print(tag, line)
