"""Mean duration of each kernel and of the gap before it, over the update loop of a rocprofv3
kernel trace (one update = fr_coop_x_kernel -> weights_gradient -> finish -> rank_draw).
usage: trace_seq.py run_kernel_trace.csv [label]"""
import collections
import csv
import sys


def main(path, label=""):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0], int(r["Start_Timestamp"]),
            int(r["End_Timestamp"])) for r in rows]
    gap, dur = collections.defaultdict(list), collections.defaultdict(list)
    lead = next((k for k in ("fr_coop_x_kernel", "pm_update_kernel", "pm_rollout_kernel", "fr_coop_kernel")
                 if any(n == k for n, _, _ in seq)), seq[0][0])
    starts = [s for n, s, e in seq if n == lead]
    for i in range(1, len(seq)):
        n, s, e = seq[i]
        if n.startswith("__amd") or seq[i - 1][0].startswith("__amd"):
            continue
        key = "%s -> %s" % (seq[i - 1][0], n)
        gap[key].append((s - seq[i - 1][2]) / 1e3)
        dur[n].append((e - s) / 1e3)
    h = len(starts) // 2   # second half of the updates (past warm-up)
    period = (starts[-1] - starts[h]) / 1e3 / max(1, len(starts) - 1 - h) if len(starts) > 2 else 0.0
    print("%s update period %.1f us" % (label, period))
    for k, v in gap.items():
        v = v[len(v) // 2:]
        print("   gap %-50s n=%3d mean %6.1f us" % (k, len(v), sum(v) / len(v)))
    for k, v in dur.items():
        v = v[len(v) // 2:]
        print("   dur %-50s n=%3d mean %6.1f us" % (k, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main(*sys.argv[1:])
