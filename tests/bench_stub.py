"""A stand-in for the engine's Trajectory that bench.py loads under MPPI_BENCH_STUB_ENGINE=1 (CPU
tests only): the bench line's assembly at N > 1 - the RCCL check, the labels, hbm.weight_reduce,
the roofline and the CPU baseline on rank 0 - runs on the CPU without a GPU.  Every number it
returns is a fixed placeholder; nothing here is measured."""
import math
import os


def comm_unique_id():
    return os.urandom(128)


class StubTrajectory:
    def __init__(self, conf, world, rank):
        self.R = conf.rollouts + 2
        self.H = int(math.ceil(conf.horison / conf.time_step))   # mppi.cpp:85
        self.world, self.rank = world, rank
        self.graph = 0
        self.timing = 0
        self.updates = self.graph_count = 0
        self.events = []

    def comm_init(self, world, rank, uid):
        assert len(uid) == 128 and world == self.world and rank == self.rank

    def comm_info(self):
        return {"nranks": self.world, "rank": self.rank, "device": self.rank,
                "pci_bus_id": "0000:%02x:00.0" % self.rank}

    def set_noise_source(self, source, seed=0):
        pass

    def set_graph(self, enable):
        self.graph = enable

    def set_forecast(self, table):
        assert table.shape == (self.H, 6)

    def set_timing(self, level):
        self.timing = level

    def update(self, x, t):
        self.updates += 1
        if self.graph and self.timing == 0:
            self.graph_count += 1
        if self.timing == 1:
            self.events.append(0.2)

    def c_update_entry(self, x):
        def fn(h, p, t):
            self.update(x, t)
            return 0
        return fn, None, None

    def synchronize(self):
        pass

    def rollout_kernel_times(self):
        out, self.events = self.events, []
        return out

    def graph_updates(self):
        return self.graph_count

    def update_info(self):
        local = self.R // self.world + (1 if self.rank < self.R % self.world else 0)
        return {"cooperative": 1, "folded_filter": 1, "objective_in_launch": 1, "tail_draws": 1, "sampling": 2,
                "rows": local + 1, "handover": -2, "wait_timeouts": 0, "wait_timeouts_total": 0,
                "fused_update": 0, "graph_updates": self.graph_count, "graph_failures": 0,
                "update_count": self.updates}

    def kernel_times(self, wait=True, detail=False):
        return [0.01, 0.2, 0.02, 0.15, 0.25, 0.19, 0.008, 0.004 if self.world > 1 else 0.0][:8 if detail else 5]

    def _check(self, st):
        assert st == 0


def creator(world, rank):
    def create(conf, dynamics, cost, device=0):
        assert device == rank
        return StubTrajectory(conf, world, rank)
    return create
