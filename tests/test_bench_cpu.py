"""bench.py's multi-GPU launch on the CPU: `python bench.py --gpus N` starts
the N rank processes itself, before any engine import or HIP call, with the rendezvous on
127.0.0.1; MPPI_BENCH_BOOTSTRAP_ONLY=1 stops each rank after the gloo bootstrap and the broadcast of
the (stand-in) RCCL unique id, so the launch is checked without a GPU.  The partition the ranks
then drive is the reference's ThreadPool split (mppi.cpp:272-307; test_abi_cpu.py covers
mppi_shard_range)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BENCH = os.path.join(os.path.dirname(HERE), "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)], env=_env(MPPI_BENCH_BOOTSTRAP_ONLY="1"),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["bootstrap_only"] and out["n_gpus"] == n
    ranks = out["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert sorted(x["local_rank"] for x in ranks) == list(range(n))   # one GPU per rank
    assert len({x["pid"] for x in ranks}) == n
    assert len({x["uid"] for x in ranks}) == 1 and len(bytes.fromhex(ranks[0]["uid"])) == 128
    assert not any(x["engine_loaded"] for x in ranks)   # nothing touched HIP before the ranks existed
    rccl = out["rccl"]   # the communicator check, on stand-ins for mppi_comm_info
    assert rccl["ranks"] == n and rccl["communicator_ranks"] == [n] * n
    assert [d["rank"] for d in rccl["devices"]] == list(range(n))
    assert len({d["pci_bus_id"] for d in rccl["devices"]}) == n


@pytest.mark.parametrize("stub", [{"MPPI_BENCH_STUB_NRANKS": "1"}, {"MPPI_BENCH_STUB_SAME_DEVICE": "1"}])
def test_bench_refuses_a_run_that_is_not_n_ranks_on_n_devices(stub):
    """A communicator whose rank count is not --gpus, or two ranks on one device: exit non-zero."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(MPPI_BENCH_BOOTSTRAP_ONLY="1", **stub),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode != 0 and "RCCL check failed" in r.stderr, (r.returncode, r.stderr[-2000:])


def test_bench_refuses_gpus_that_disagree_with_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def _stub_line(args, **env):
    r = subprocess.run([sys.executable, BENCH] + args, env=_env(MPPI_BENCH_STUB_ENGINE="1", **env),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    return json.loads(lines[0])


def test_bench_line_schema_at_two_ranks():
    """The N > 1 line on a stand-in engine (tests/bench_stub.py): rank 0 times
    the CPU baseline on the whole job's workload after the timed loop, the weight reduce is reported
    without the cost all-reduce (timed beside it), and the RCCL check and labels hold."""
    d = _stub_line(["--gpus", "2", "--steps", "3", "--warmup", "1", "--samples-per-gpu", "64", "--horizon-steps", "8",
                    "--cpu-updates", "2", "--cpu-warmup", "1"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "hbm", "rccl"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["samples"] == 128
    assert d["rccl"]["communicator_ranks"] == [2, 2]
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["timed_updates"] == 2 and "2-rank job" in cb["sample"]
    assert "128x8" in cb["sample"]   # the total workload, not one rank's share
    wr = d["hbm"]["weight_reduce"]
    assert wr["cost_allreduce_ms"] > 0 and "not including it" in wr["note"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    assert not d["config"]["workload"].startswith("BASELINE")   # 128 x 8 is no BASELINE config


def test_bench_graph_mode_times_every_update_as_the_graph():
    """--graph 1 (with --comm1: the sharded path through a one-rank communicator): the timed loop
    records no timing events, so every timed update can replay the graph (graph_updates_timed ==
    steps); the rollout launch is timed over eager updates after the loop."""
    d = _stub_line(["--steps", "5", "--warmup", "2", "--samples-per-gpu", "64", "--horizon-steps", "8", "--graph", "1",
                    "--comm1", "1", "--no-cpu-baseline"])
    assert d["engine"]["graph_updates_timed"] == 5
    assert d["config"]["comm1"] == 1 and "one-rank RCCL" in d["config"]["workload"]
    assert "eager updates after the timed (graph) loop" in d["roofline"]["launch_time_source"]
    assert d["kernel_ms"]["rollout_launch_samples"] > 0


def test_bench_workload_labels():
    """config.workload names the BASELINE config by the run's total shape."""
    sys.path.insert(0, os.path.dirname(BENCH))
    import bench
    assert bench.workload_label(False, 4096, 64, 0, 1, -1) == "BASELINE configs[2]: "
    assert bench.workload_label(False, 8192, 64, 0, 2, -1).startswith("BASELINE configs[2]'s 4096 x 64 per GPU")
    assert bench.workload_label(False, 32768, 64, 0, 8, -1) == "BASELINE configs[3]: "
    assert bench.workload_label(False, 32768, 64, 0, 1, -1) == "BASELINE configs[3]: "
    assert bench.workload_label(False, 65536, 128, 10, 8, 1) == "BASELINE configs[4]: "
    assert "eager" in bench.workload_label(False, 65536, 128, 10, 8, 0)
    assert bench.workload_label(False, 16384, 64, 0, 4, -1).startswith("BASELINE configs[2]'s")
    assert bench.workload_label(False, 8192, 128, 10, 1, 1) == ""
    assert bench.workload_label(True, 1024, 32, 0, 1, -1) == "BASELINE configs[1]: "
