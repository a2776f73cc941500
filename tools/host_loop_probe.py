"""Host turnaround probe (run on the GPU box with MPPI_HOST_TRACE=1): the 4096x64 update loop
driven three ways - through Trajectory.update, through the raw ctypes entry point, and as bench.py
drives it (timing level 1 every 4th update) - printing ms/update; the engine prints its host
stamps when each handle closes."""
import os
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import assistedmanipulation_amd as am  # noqa: E402
from assistedmanipulation_amd import abi  # noqa: E402


def make():
    conf = am.frankaridgeback_configuration(rollouts=4096, horison=0.64, keep_best_rollouts=20)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    return t


def run(mode, n=int(os.environ.get("PROBE_N", "200"))):
    # PROBE_WARM: untimed updates first (the GPU's warm-up takes ~120 updates, tools/ramp_probe.py)
    warm = int(os.environ.get("PROBE_WARM", "10"))
    t = make()
    x = am.huddled_state()
    for j in range(warm):
        t.update(x, 0.05 * j)
    f, h, ptr = t._L.mppi_update, t._h, t._state_ptr
    t._state_buf[:] = x
    j = warm
    t0 = time.perf_counter()
    for i in range(n):
        if mode == "wrapper":
            t.update(x, 0.05 * j)
        elif mode == "raw":
            f(h, ptr, 0.05 * j)
        else:
            s = i % 4 == 0
            if s:
                t.set_timing(1)
            t.update(x, 0.05 * j)
            if s:
                t.set_timing(0)
        j += 1
    t.synchronize()
    dt = (time.perf_counter() - t0) / n
    print("%-8s %.4f ms/update" % (mode, dt * 1e3), flush=True)
    t.close()


for m in sys.argv[1:] or ["wrapper", "raw", "bench"]:
    run(m)
