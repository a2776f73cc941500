"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo).

The engine shards rollouts with mppi_shard_range and exchanges exactly two buffers per update:
an all-reduce(sum) of the zero-padded cost vector [R] and of the partial gradient [C x H]
(engine.cpp mppi_update).  Here each gloo rank runs the oracle in the same sharded
mode — its own shard's rollouts, the two sums through torch.distributed — and must reproduce the
unsharded update.  Also checks the bench bootstrap (unique-id broadcast)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import ctypes as C

    import assistedmanipulation_amd as am   # engine library before torch
    from oracle import oracle as O
    import torch
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        conf = am.frankaridgeback_configuration(rollouts=62, horison=0.16, keep_best_rollouts=10, threads=2)
        cc, keep = conf.to_c()
        d, c = am.FrankaRidgebackDynamics().descriptor(), am.AssistedManipulation().descriptor()
        sharded = O.OracleTrajectory(cc, d, c)
        full = O.OracleTrajectory(cc, d, c)
        R = sharded.R
        b, e = am.shard_range(R, world, rank)

        def allreduce(ptr, n):
            arr = np.ctypeslib.as_array(ptr, shape=(n,))
            t = torch.from_numpy(arr)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

        sharded.set_shard(b, e, allreduce)
        table = am.constant_forecast(sharded.H)
        sharded.set_forecast(table)
        full.set_forecast(table)
        rng = np.random.default_rng(2024)   # same stream on every rank
        sd = np.sqrt(np.diag(conf.covariance))
        x = am.huddled_state()
        worst = 0.0
        for j in range(4):
            t = 0.05 * j
            n = full.noise_draws(t)
            eps = rng.standard_normal((n, 12)) * sd
            for tr in (sharded, full):
                tr.inject_noise(eps)
                tr.update(x, t)
            np.testing.assert_allclose(sharded.costs(), full.costs(), rtol=1e-13, atol=0)
            assert int(np.nanargmin(sharded.costs())) == int(np.nanargmin(full.costs()))
            np.testing.assert_allclose(sharded.weights(), full.weights(), rtol=0, atol=1e-15)
            np.testing.assert_allclose(sharded.optimal_control(), full.optimal_control(), rtol=0, atol=1e-12)
            worst = max(worst, float(np.abs(sharded.optimal_control() - full.optimal_control()).max()))
        # bench.py bootstrap: rank 0's 128-byte id reaches every rank
        uid = [bytes(range(128)) if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        assert uid[0] == bytes(range(128))
        dist.barrier()
        q.put((rank, "ok", worst, (b, e)))
    except Exception as ex:   # report to the parent
        import traceback
        q.put((rank, "fail", traceback.format_exc(), None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_two_rank_sharded_update_equals_unsharded():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, status, info, span in results:
        assert status == "ok", info
    spans = sorted(r[3] for r in results)
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == 64
