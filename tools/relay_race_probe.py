"""Repeatability probe for the rows left over (a GPU diagnostic, not a test): the graph-test sequence
(tests/test_gpu_scale.py::test_graph_path_equals_eager_launches: shifts, a state change, a
standalone filter() between updates) run on several handles that must agree bit for bit - relay in
one workgroup (MPPI_RELAY_K=1) and over two (K=2), eager and captured - and every mismatching
rollout printed with the update, the launch row it sat in and whether that row is a relay row.

usage: python tools/relay_race_probe.py [--rollouts 1000] [--reps 3] [--ks 1,2,2] [--graph 0,0,0]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import assistedmanipulation_amd as am  # noqa: E402
from assistedmanipulation_amd import abi  # noqa: E402


def run(rollouts, horison, k, graph, times, interrupt):
    os.environ["MPPI_RELAY_K"] = str(k)
    conf = am.frankaridgeback_configuration(rollouts=rollouts, horison=horison, keep_best_rollouts=20, threads=8)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    t.set_graph(graph)
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    x = am.huddled_state()
    rec = []
    for j, tm in enumerate(times):
        if j == 5:
            x = x.copy()
            x[12 + 4] = 0.3
        t.update(x, tm)
        info = t.update_info()
        rec.append((t.noise().copy(), t.costs().copy(), info["rows"], info["wait_timeouts"]))
        if j in interrupt:
            t.get_optimal_total_cost()
    return rec


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rollouts", type=int, default=1000)
    p.add_argument("--horison", type=float, default=0.64)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--ks", default="1,2,2")
    p.add_argument("--graph", default="0,0,1")
    a = p.parse_args()
    times = [0.0, 0.05, 0.07, 0.12, 0.12, 0.17, 0.22, 0.27, 0.32, 0.37, 0.40, 0.45, 0.50, 0.55]
    interrupt = {6, 9, 12}
    ks = [int(v) for v in a.ks.split(",")]
    gs = [int(v) for v in a.graph.split(",")]
    bad = 0
    for rep in range(a.reps):
        runs = [run(a.rollouts, a.horison, k, g, times, interrupt) for k, g in zip(ks, gs)]
        for i in range(1, len(runs)):
            for j, (u, v) in enumerate(zip(runs[0], runs[i])):
                nz = np.array_equal(u[0], v[0], equal_nan=True)
                cz = np.flatnonzero(~((u[1] == v[1]) | (np.isnan(u[1]) & np.isnan(v[1]))))
                if len(cz) or not nz:
                    bad += 1
                    rows = u[2]
                    xbase = (rows // 16) * 16
                    print("rep %d run %d (K=%d graph=%d) update %d: rows %d/%d timeouts %d/%d, cost mismatch at %s "
                          "(relay rows from %d), rel %s, noise equal %s" %
                          (rep, i, ks[i], gs[i], j, u[2], v[2], u[3], v[3], cz.tolist(), xbase,
                           [float(abs(u[1][c] - v[1][c]) / abs(u[1][c])) for c in cz[:4]],
                           nz), flush=True)
        print("rep %d done" % rep, flush=True)
    print("mismatching updates:", bad)


if __name__ == "__main__":
    main()
