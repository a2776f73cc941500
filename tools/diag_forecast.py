"""Diagnose device-forecast update parity: forecast values vs the oracle's, per update."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import assistedmanipulation_amd as am
from oracle import oracle as O
from helpers import fr_pair, step_both

cfg = am.kalman_forecast_configuration(0.005, 0.3, 2)
conf, dev, orc, sd = fr_pair(S=128, horison=0.32, forecast=False)
dev.attach_forecast(cfg)
fc = O.OracleForecast(cfg)
rng = np.random.default_rng(17)
x = am.huddled_state()
obs_t = 0.0
for j in range(3):
    t = 0.05 * j
    while obs_t <= t + 1e-12:
        w = np.array([20 + 10 * np.sin(3 * obs_t), 5 * np.cos(obs_t), 2.0, 0.1, 0.0, -0.1]) + rng.normal(0, 0.5, 6)
        dev.observe_wrench(w, obs_t)
        fc.observe(w, obs_t)
        for q in (0.001, 0.002, 0.003, 0.004):
            dev.observe_time(obs_t + q)
            fc.observe_time(obs_t + q)
        obs_t += 0.005
    tab = fc.table(t, conf.time_step, dev.H)
    dtab = np.array([dev.forecast(t + k * conf.time_step) for k in range(dev.H)])
    print("upd", j, "forecast max diff", np.max(np.abs(tab - dtab)), "rows nonzero", int(np.sum(np.any(tab != 0, axis=1))))
    orc.set_forecast(tab)
    step_both(dev, orc, x, t, rng, sd)
    cd, co = dev.costs(), orc.costs()
    rel = np.abs(cd - co) / np.maximum(np.abs(co), 1)
    print("   cost rel max", rel.max(), "argmax", int(np.argmax(rel)), "n bad", int(np.sum(rel > 1e-11)))
