"""The engine's sharded update in two processes (missing #1): two fresh child
processes on device 0 each hold a phase-split shard (mppi_set_shard(2, r)) and exchange the R + 1
costs and the partial gradient over gloo between the phases (tests/mp_shard_worker.py), against one
unsharded handle in this process.  Replaces the reference's ThreadPool split
(concurrency.hpp:187-216, mppi.cpp:272-307) with processes, as one rank per GPU would run it; the
same device is used twice because a gpurun box has one GPU (RCCL refuses two ranks on one device,
so the exchange goes over gloo on the host).  Device Philox: draws are keyed by global rollout."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("S,horison,updates", [(4096, 0.64, 3)])
def test_two_process_shards_equal_unsharded(S, horison, updates, tmp_path):
    world, port = 2, _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / ("rank%d.npz" % r))
        outs.append(out)
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_shard_worker.py"), out, str(S),
                                       str(horison), str(updates)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=150)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d rc %d:\n%s" % (r, p.returncode, logs[r][-3000:])
    res = [dict(np.load(o)) for o in outs]
    assert res[0]["pid"] != res[1]["pid"] and int(res[0]["pid"]) != os.getpid()

    conf = am.frankaridgeback_configuration(rollouts=S, horison=horison, keep_best_rollouts=20, threads=8)
    single = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    single.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    single.set_forecast(am.constant_forecast(single.H))
    x = am.huddled_state()
    worst = (0.0, 0.0, 0.0)
    for j in range(updates):
        single.update(x, 0.05 * j)
        cu, uu, wu, full = single.costs(), single.get_optimal_rollout(), single.get_weights(), single.noise()
        delta = np.nanmax(cu) - np.nanmin(cu)
        for r, d in enumerate(res):
            b, e = (int(v) for v in d["shard"])
            assert (b, e) == am.shard_range(single.R, world, r)
            k = max(2 - b, 0)   # rollout 1 carries -U*: its bits follow the gradient's summation order
            np.testing.assert_array_equal(d["noise_%d" % j][k:], full[b:e][k:], err_msg="update %d rank %d noise" % (j, r))
            cs = d["costs_%d" % j]
            if j == 0:   # both sides start from U* = 0: identical bits
                np.testing.assert_array_equal(cs, cu)
            bad = np.abs(cs - cu) > 1e-11 * (delta + np.abs(cu))
            assert not bad.any(), "update %d rank %d rollout %d: %r vs %r" % (j, r, int(np.argmax(bad)),
                                                                              cs[np.argmax(bad)], cu[np.argmax(bad)])
            du = np.max(np.abs(d["u_%d" % j] - uu))
            dw = np.max(np.abs(d["w_%d" % j] - wu))
            assert du <= 1e-12 and dw <= 1e-15, (j, r, du, dw)
            assert int(d["argmin_%d" % j]) == single.argmin()
            worst = tuple(max(a, v) for a, v in zip(worst, (np.nanmax(np.abs(cs - cu)) / delta, du, dw)))
    assert all(int(d["update_count"]) == updates for d in res)
    print("two processes vs one handle, worst (cost error / Delta, U* abs, weights abs):", worst)
