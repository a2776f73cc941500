"""Where the time between updates goes, from one rocprofv3 run with --kernel-trace and
--hip-runtime-trace (csv): each kernel dispatch is joined to the HIP call that launched it by its
correlation id, and for every launch of KERNEL (a substring, default the rollout kernel) after
the first `skip` it prints the mean of
  prev_end -> call   the end of the previous kernel on the device to the launch call's start
                     (the host: seeing the publish, returning, the caller's loop, phase 1)
  call               the launch call itself (hipLaunchKernel / hipExtLaunchKernel ...)
  call_end -> start  the call's return to the kernel's start on the device (dispatch)
  prev_end -> start  the whole gap
usage: launch_latency.py RUN_DIR [KERNEL] [skip]"""
import csv
import glob
import os
import sys


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(d, kname="fr_coop_x_kernel", skip=20):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    if not kt or not ht:
        sys.exit("need *kernel_trace.csv and *hip_api_trace.csv under %s" % d)
    ks = sorted(rows(kt[0]), key=lambda r: int(r["Start_Timestamp"]))
    api = {r["Correlation_Id"]: r for r in rows(ht[0])}
    out = []
    for i, k in enumerate(ks):
        if kname not in k["Kernel_Name"] or i == 0:
            continue
        a = api.get(k["Correlation_Id"])
        if a is None:
            continue
        prev_end = int(ks[i - 1]["End_Timestamp"])
        cs, ce = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        s = int(k["Start_Timestamp"])
        out.append((cs - prev_end, ce - cs, s - ce, s - prev_end, ks[i - 1]["Kernel_Name"][:40], a["Function"]))
    out = out[skip:]
    if not out:
        sys.exit("no launches of %s" % kname)
    n = len(out)
    mean = [sum(o[j] for o in out) / n / 1e3 for j in range(4)]
    print("%s: %d launches (after %d), previous kernel %s, call %s" % (kname, n, skip, out[-1][4], out[-1][5]))
    print("  prev_end -> call %.2f us, call %.2f us, call_end -> start %.2f us, prev_end -> start %.2f us" % tuple(mean))
    med = [sorted(o[j] for o in out)[n // 2] / 1e3 for j in range(4)]
    print("  medians: prev_end -> call %.2f us, call %.2f us, call_end -> start %.2f us, prev_end -> start %.2f us" % tuple(med))
    srt = sorted(o[3] for o in out)
    print("  prev_end -> start p10 %.2f p50 %.2f p90 %.2f us" % (srt[n // 10] / 1e3, srt[n // 2] / 1e3, srt[9 * n // 10] / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fr_coop_x_kernel", int(sys.argv[3]) if len(sys.argv) > 3 else 20)
