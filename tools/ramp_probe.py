"""Cold-start probe (GPU box): why the driver's 20-update bench runs slower than the steady state.
Creates the 4096x64 handle as bench.py does, then times every update of the first N one by one
(host perf_counter around Trajectory.update, which returns once U* is published) and prints the
mean per bucket of 10, with the GPU's current shader / memory clock levels read from sysfs (read
only) before the first update, after 25 and after N.  Optional argv[1]: N (default 600);
argv[2]: a pause in ms after the first 25 updates (default 0), to see the clocks fall back;
argv[3] = "rehandle": afterwards a second handle (U* from zero again) on the now-busy GPU, its
first 60 updates timed the same way (hardware warm-up vs the optimisation's own state), and
per-update rollout-kernel times (HIP events, timing level 1) of both handles' first updates."""
import glob
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np  # noqa: E402
import assistedmanipulation_amd as am  # noqa: E402
from assistedmanipulation_amd import abi  # noqa: E402


def clocks():
    out = []
    for card in sorted(glob.glob("/sys/class/drm/card*/device"))[:16]:
        try:
            s = open(card + "/pp_dpm_sclk").read().split("\n")
            m = open(card + "/pp_dpm_mclk").read().split("\n")
        except OSError:
            continue
        cur = [l for l in s if l.strip().endswith("*")]
        curm = [l for l in m if l.strip().endswith("*")]
        out.append("%s sclk %s mclk %s" % (card.split("/")[-2], cur[0].strip() if cur else "?", curm[0].strip() if curm else "?"))
    return "; ".join(out) if out else "sysfs clocks unreadable"


def make():
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.64, keep_best_rollouts=20)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    return t


def kernel_series(t, x, n, j0=0):
    """rollout-kernel ms of each of n updates (timing level 1 on every update)"""
    ks = []
    for j in range(n):
        t.rollout_kernel_times()
        t.set_timing(1)
        t.update(x, 0.05 * (j0 + j))
        t.set_timing(0)
        v = t.rollout_kernel_times()
        ks.append(v[-1] if len(v) else float("nan"))
    return np.array(ks)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    pause = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    rehandle = len(sys.argv) > 3 and sys.argv[3] == "rehandle"
    t = make()
    x = am.huddled_state()
    print("before:", clocks(), flush=True)
    dts = np.zeros(n)
    for j in range(n):
        if j == 25:
            print("after 25:", clocks(), flush=True)
            if pause > 0:
                time.sleep(pause * 1e-3)
        a = time.perf_counter()
        t.update(x, 0.05 * j)
        dts[j] = time.perf_counter() - a
    t.synchronize()
    print("after %d:" % n, clocks(), flush=True)
    for b in range(0, n, 10):
        print("updates %3d-%3d  %.4f ms" % (b, b + 9, 1e3 * dts[b:b + 10].mean()), flush=True)
    print("first 5 %.4f, 5-25 %.4f, last 200 %.4f ms" % (1e3 * dts[:5].mean(), 1e3 * dts[5:25].mean(),
                                                       1e3 * dts[-200:].mean()), flush=True)
    if rehandle:
        k1 = kernel_series(t, x, 60, n)
        t.close()
        t2 = make()
        d2 = np.zeros(60)
        for j in range(60):
            a = time.perf_counter()
            t2.update(x, 0.05 * j)
            d2[j] = time.perf_counter() - a
        k2 = kernel_series(t2, x, 60, 60)
        t2.close()
        t3 = make()
        k3 = kernel_series(t3, x, 200)
        t3.close()
        for b in range(0, 60, 10):
            print("second handle updates %2d-%2d  %.4f ms" % (b, b + 9, 1e3 * d2[b:b + 10].mean()), flush=True)
        print("rollout kernel ms: first handle after %d: %.4f; second handle updates 60-119: %.4f" % (n, k1.mean(), k2.mean()))
        for b in range(0, 200, 20):
            print("third handle rollout kernel updates %3d-%3d  %.4f ms" % (b, b + 19, k3[b:b + 20].mean()), flush=True)
        return
    t.close()


if __name__ == "__main__":
    main()
