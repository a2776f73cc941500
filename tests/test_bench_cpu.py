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
