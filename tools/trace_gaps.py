"""Average duration of each kernel and the mean update period from a rocprofv3 kernel trace.
usage: trace_gaps.py run_kernel_trace.csv [label]"""
import collections
import csv
import sys


def main(path, label=""):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    dur = collections.defaultdict(list)
    starts = []
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name[:name.find("(")] if "(" in name else name
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if name.startswith("void sample_kernel"):
            starts.append(int(r["Start_Timestamp"]))
    period = (starts[-1] - starts[len(starts) // 2]) / 1e3 / max(1, len(starts) - 1 - len(starts) // 2)
    print("%s update period %.1f us" % (label, period))
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("   %-45s n=%3d avg %7.1f us" % (n[:45], len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main(*sys.argv[1:])
