"""One rank of the two-process sharded engine test (tests/test_gpu_multiproc.py; VERDICT r05 item
7): a phase-split shard of the rollouts (mppi_set_shard(world, rank), the reference's ThreadPool
partition mppi.cpp:272-307) on the GPU, the two exchanges between the phases - the R + 1 costs
(mppi_device_costs_count) and the partial gradient - summed across the processes over gloo, as
concurrency.hpp:187-216's threads hand their shares to the one optimise().

    python tests/mp_shard_worker.py OUT.npz S HORISON UPDATES   (RANK / WORLD_SIZE / MASTER_* in the env)
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import assistedmanipulation_amd as am   # noqa: E402  (the engine library before torch)
from assistedmanipulation_amd import abi  # noqa: E402


def main():
    out, S, horison, updates = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipDeviceSynchronize.argtypes = []
    conf = am.frankaridgeback_configuration(rollouts=S, horison=horison, keep_best_rollouts=20, threads=8)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation(), device=0)
    assert t is not None
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    t.set_shard(world, rank)
    n_costs = t.device_costs_count()
    assert n_costs == t.R + 1   # the costs and slot R (the ranks' in-launch wait timeouts)
    HC = t.H * t.C

    def allreduce(ptr, n):   # device -> host, gloo sum across the processes, host -> device
        buf = np.zeros(n)
        assert hip.hipDeviceSynchronize() == 0
        assert hip.hipMemcpy(buf.ctypes.data, ptr, n * 8, 2) == 0
        tb = torch.from_numpy(buf)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        assert hip.hipMemcpy(ptr, buf.ctypes.data, n * 8, 1) == 0

    x = am.huddled_state()
    res = {}
    b, e = am.shard_range(t.R, world, rank)
    for j in range(updates):
        tm = 0.05 * j
        t.update_phase1(x, tm)
        allreduce(t.device_costs_ptr(), n_costs)
        t.update_phase2()
        allreduce(t.device_gradient_ptr(), HC)
        t.update_phase3(tm)
        res["costs_%d" % j] = t.costs()
        res["u_%d" % j] = t.get_optimal_rollout()
        res["w_%d" % j] = t.get_weights()
        res["argmin_%d" % j] = np.array(t.argmin())
        res["noise_%d" % j] = t.noise()[b:e]
    res["pid"] = np.array(os.getpid())
    res["shard"] = np.array([b, e])
    res["update_count"] = np.array(t.get_update_count())
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()
    t.close()


if __name__ == "__main__":
    main()
