"""Device-forecast update parity under simpler event streams (isolates the failing piece)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import assistedmanipulation_amd as am
from oracle import oracle as O
from helpers import fr_pair, step_both


def run(name, cfg, observe_between):
    conf, dev, orc, sd = fr_pair(S=128, horison=0.32, forecast=False)
    dev.attach_forecast(cfg)
    fc = O.OracleForecast(cfg)
    rng = np.random.default_rng(17)
    x = am.huddled_state()
    out = []
    for j in range(3):
        t = 0.05 * j
        if j == 0 or observe_between:
            w = np.array([20.0, 5.0, 2.0, 0.1, 0.0, -0.1]) * (1 + 0.1 * j)
            dev.observe_wrench(w, t)
            fc.observe(w, t)
        orc.set_forecast(fc.table(t, conf.time_step, dev.H))
        step_both(dev, orc, x, t, rng, sd)
        cd, co = dev.costs(), orc.costs()
        out.append(float(np.max(np.abs(cd - co) / np.maximum(np.abs(co), 1))))
    print("%-28s %s" % (name, " ".join("%.2e" % v for v in out)))


run("locf obs-once", am.locf_forecast_configuration(horison=10.0), False)
run("locf obs-each", am.locf_forecast_configuration(horison=10.0), True)
run("kalman1 obs-once", am.kalman_forecast_configuration(0.005, 0.3, 1), False)
run("kalman1 obs-each", am.kalman_forecast_configuration(0.005, 0.3, 1), True)


def host_steps(table, H, gamma=1.0):
    """build_steps (engine.cpp) in numpy from a forecast table, AssistedManipulation defaults."""
    a = am.AssistedManipulation().configuration
    out = np.zeros((H, 8))
    for k in range(H):
        tg = np.clip(a.trajectory_target_scale * table[k, :3], -a.trajectory_target_maximum, a.trajectory_target_maximum)
        tt = tg @ tg
        d = np.sqrt(tt)
        pc = a.trajectory_position_cost
        vt = min(max(np.exp(a.trajectory_velocity_dropoff * d) - 1, a.trajectory_velocity_minimum), a.trajectory_velocity_maximum)
        out[k] = [tg[0], tg[1], tg[2], tt, (pc.constant_cost + pc.linear_cost * abs(d)) + pc.quadratic_cost * d * d, vt,
                  gamma ** k, 1.0 if (a.has_forecast and d > a.trajectory_position_threshold) else 0.0]
    return out


cfg = am.kalman_forecast_configuration(0.005, 0.3, 1)
conf, dev, orc, sd = fr_pair(S=128, horison=0.32, forecast=False)
dev.attach_forecast(cfg)
fc = O.OracleForecast(cfg)
rng = np.random.default_rng(17)
x = am.huddled_state()
w = np.array([20.0, 5.0, 2.0, 0.1, 0.0, -0.1])
dev.observe_wrench(w, 0.0)
fc.observe(w, 0.0)
for j in range(3):
    t = 0.05 * j
    tab = fc.table(t, conf.time_step, dev.H)
    orc.set_forecast(tab)
    step_both(dev, orc, x, t, rng, sd)
    sc = dev.step_constants()
    ref = host_steps(tab, dev.H)
    bad = np.nonzero(np.any(np.abs(sc - ref) > 1e-12 * np.maximum(1, np.abs(ref)), axis=1))[0]
    print("upd", j, "step-constant rows differing:", bad[:10], "max", np.max(np.abs(sc - ref)))
    if len(bad):
        k = bad[0]
        print("   dev", sc[k], "\n   ref", ref[k], "\n   tab", tab[k], "dev fc", dev.forecast(t + k * conf.time_step))
