#!/usr/bin/env python3
"""MPPI rollout throughput on MI355X — BASELINE.json's metric.

A "step" is one mppi::Trajectory::update() (reference src/controller/mppi.cpp:154-187, its own
timing boundary) with the reference's cadence: updates at t = 0.05 j (5-step shift), keep-best 20,
device Philox noise.  value = samples x horizon x ranks / (max-over-ranks seconds per update).

Workloads (BASELINE.json configs):
  frankaridgeback (default)  FrankaRidgeback Pinocchio dynamics + full AssistedManipulation cost,
                             4096 samples x 64 steps per GPU (configs[2]; configs[3] at N = 8);
                             --horizon-steps 128 --smoothing 10 for configs[4]'s shape
  point_mass                 the analytic bring-up plugin, 1024 x 32 (configs[1])

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload point_mass]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N rank processes
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each) before anything imports the
engine or touches HIP, and exits with their status; under torch.distributed.run WORLD_SIZE must
equal --gpus.  Each rank rolls out its contiguous share of the rollouts (mppi.cpp:272-307's
partition, mppi_shard_range) and the engine all-reduces the costs and the partial gradient over
RCCL; rank 0 prints the one JSON line.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

am = abi = None   # the engine package, imported by run() - after the rank processes exist

SAMPLES_PER_GPU = 4096
HORIZON_STEPS = 64        # 0.64 s at dt = 0.01
KEEP_BEST = 20
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 vector (= fp64 matrix) peak, AMD spec; the rollout is fp64 VALU
# Algorithmic FLOPs of one rollout-step of the minimal arithmetic the device executes
# (world-frame zero-bias dynamics + kinematics + default cost), counted by the oracle's
# FLOP-counting scalar (tests/test_oracle_cpu.py::test_flop_count_constant pins these values):
# the cost part (get_cost) and the rest (dynamics + kinematics).
FLOPS_PER_ROLLOUT_STEP = 6518.0
FLOPS_COST_PER_ROLLOUT_STEP = 690.0
FLOPS_DYN_PER_ROLLOUT_STEP = FLOPS_PER_ROLLOUT_STEP - FLOPS_COST_PER_ROLLOUT_STEP
# SURVEY §8(d)'s algorithmic HBM bytes per rollout-step: the eps column written once when sampled and
# read once by the weight reduce, 2 C x sizeof (fp32 in the survey; the device stores fp64 eps).
BYTES_SURVEY_FR = 2 * 12 * 8.0    # 192 B (FrankaRidgeback, C = 12)
BYTES_SURVEY_PM = 2 * 3 * 8.0     # 48 B (point mass, C = 3)
# What the device's rollout launch moves beyond that: it reads the eps column (96 B),
# and the cooperative kernel writes a 768-B step record that the objective reads back.
BYTES_EPS_FR = 96.0
BYTES_REC = 768.0   # the stored step record (kernels.hpp FR_REC; 336 B until r05)
EV_EVERY = 8   # timed updates per rollout-kernel event sample
EV_GRAPH = 16  # --graph 1: eager updates after the timed loop whose rollout launches are timed
PMC_JSON = os.path.join(HERE, "profiles", "r06", "final", "pmc_rollout.json")
PMC_WG_JSON = os.path.join(HERE, "profiles", "r06", "final", "pmc_weights.json")   # weights_gradient_kernel's traffic
PMC_PM_JSON = os.path.join(HERE, "profiles", "r06", "final", "pmc_pm.json")      # pm_update_kernel's traffic


def recorded_label(path):
    """The PMC traffic beside the live timings is recorded, not measured in this run: name the
    profile file and the kernel build it was collected on (its 'recorded' field)."""
    try:
        with open(path) as f:
            rec = json.load(f).get("recorded", "")
    except (OSError, ValueError):
        rec = ""
    return "recorded (not this run): %s%s" % (os.path.relpath(path, HERE), ", " + rec if rec else "")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 200 timed updates (~60 ms): the last update's filter(), finished inside the timed region by
    # the closing synchronize (~0.18 ms alone), is spread over the steady-state updates
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", choices=("frankaridgeback", "point_mass"), default="frankaridgeback")
    p.add_argument("--samples-per-gpu", type=int, default=None, help="4096 (frankaridgeback) / 1024 (point_mass)")
    p.add_argument("--horizon-steps", type=int, default=None,
                   help="H (dt = 0.01); 64 = configs[2]/[3], 128 = configs[4]; 32 for point_mass")
    p.add_argument("--smoothing", type=int, default=0, help="Savitzky-Golay window (order 1); 10 = configs[4]")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the CPU baseline (0: the CPU share this process may use)")
    p.add_argument("--cpu-updates", type=int, default=50, help="timed CPU updates (median / p90), BASELINE.md §2")
    p.add_argument("--cpu-warmup", type=int, default=5, help="untimed CPU warm-up updates, BASELINE.md §2")
    p.add_argument("--graph", type=int, default=-1,
                   help="1: the hipGraph update path (mppi_set_graph), 0: eager launches, -1: the engine's default")
    p.add_argument("--comm1", type=int, default=0,
                   help="1 (N = 1 only): run the sharded update through a one-rank RCCL communicator "
                        "(mppi_comm_init(1, 0)): the cost and gradient all-reduces, and with --graph 1 the "
                        "captured graph with RCCL's nodes, timed on one GPU")
    a = p.parse_args()
    pm = a.workload == "point_mass"
    if a.samples_per_gpu is None:
        a.samples_per_gpu = 1024 if pm else SAMPLES_PER_GPU
    if a.horizon_steps is None:
        a.horizon_steps = 32 if pm else HORIZON_STEPS
    return a


def cpu_share():
    """CPUs this process may run on: its affinity mask, capped by OMP_NUM_THREADS (the GPU box sets
    it to the per-GPU CPU share, 16) - not os.cpu_count(), which counts the whole host."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def time_oracle(libpath, conf, dyn, cost, updates, warmup, compat_uint8=0, forecast=True):
    """Median / p90 seconds per Trajectory::update of the oracle (its own steady_clock boundary,
    mppi.cpp:161-184) over `updates` timed updates after `warmup` untimed ones, t = 0.05 j."""
    from oracle import oracle as O
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, dyn.descriptor(), cost.descriptor(), lib_path=libpath, compat_uint8=compat_uint8)
    orc.set_noise_source(False, 12345)
    if forecast:
        orc.set_forecast(am.constant_forecast(orc.H))
    x = np.asarray(conf.initial_state, dtype=np.float64)
    for j in range(warmup):
        orc.update(x, 0.05 * j)
    durs = []
    for j in range(warmup, warmup + updates):
        orc.update(x, 0.05 * j)
        durs.append(orc.update_duration())
    return float(np.median(durs)), float(np.percentile(durs, 90)), orc.H


def cpu_baseline(args, pm, world=1):
    """The oracle (fp64 restatement of the reference's CPU mppi.cpp path, Pinocchio-order
    arithmetic, contiguous-block thread partition of mppi.cpp:272-307) on this host, g++ -O3
    -march=native: the bench's workload at the process's CPU share (WIDE indices: R > 255 hangs
    the reference's uint8 loops), and configs[0] (128 x 32, one thread, the reference's own uint8
    index semantics); median and p90 over --cpu-updates timed updates each."""
    from oracle import oracle as O
    try:
        libpath = O.build(native=True)   # g++ -O3 -march=native on the GPU box host
    except Exception:
        libpath = O.LIB_PATH
    threads = args.cpu_threads or cpu_share()
    S, H = args.samples_per_gpu * world, args.horizon_steps   # the whole job's workload
    # bounded: the configured updates at configs[2]'s size, scaled down for larger workloads (about
    # 10-30 s of CPU work at 16 threads), at least 3 timed and 1 warm-up
    scale = (4096.0 * 64) / (S * H)
    updates = args.cpu_updates if scale >= 1 else max(3, int(args.cpu_updates * scale))
    warm = args.cpu_warmup if scale >= 1 else max(1, int(args.cpu_warmup * scale))
    if pm:
        conf = am.point_mass_configuration(rollouts=S, horison=H * 0.01, keep_best_rollouts=KEEP_BEST)
        conf.threads = threads
        dyn, cost = am.PointMassDynamics(), am.QuadraticCost()
    else:
        conf = am.frankaridgeback_configuration(rollouts=S, horison=H * 0.01, keep_best_rollouts=KEEP_BEST,
                                                threads=threads)
        dyn, cost = am.FrankaRidgebackDynamics(), am.AssistedManipulation()
    med, p90, Ho = time_oracle(libpath, conf, dyn, cost, updates, warm, forecast=not pm)
    nproc = os.cpu_count() or 0
    out = {"value": S * Ho / med, "unit": "rollout-steps/s", "cores": threads, "kind": "port",
           "median_s_per_update": med, "p90_s_per_update": p90, "warmup_updates": warm,
           "timed_updates": updates, "process_cpu_share": cpu_share(), "host_nproc": nproc,
           "cpu_model": cpu_model(),
           "sample": "%d warm-up + %d timed updates of the %dx%d %s workload (BASELINE.md §2), "
                     "oracle/mppi_oracle.cpp fp64, g++ -O3 -march=native, %d threads: the process's CPU share "
                     "(affinity mask capped by OMP_NUM_THREADS), not the host's nproc %d, which the GPU box "
                     "shares between its GPUs; host %s" % (
                         warm, updates, S, Ho, "point-mass" if pm else "FrankaRidgeback",
                         threads, nproc, cpu_model())}
    if not pm:   # configs[0]: the reference's own plumbing case, single thread, uint8 indices
        c0 = am.frankaridgeback_configuration(rollouts=128, horison=0.32, keep_best_rollouts=KEEP_BEST, threads=1)
        m0, q0, H0 = time_oracle(libpath, c0, am.FrankaRidgebackDynamics(), am.AssistedManipulation(),
                                 args.cpu_updates, args.cpu_warmup, compat_uint8=1)
        out["configs0"] = {"value": 128 * H0 / m0, "unit": "rollout-steps/s", "cores": 1,
                           "median_s_per_update": m0, "p90_s_per_update": q0,
                           "warmup_updates": args.cpu_warmup, "timed_updates": args.cpu_updates,
                           "workload": "128 x 32 FrankaRidgeback, single thread, uint8 index semantics (BASELINE configs[0])"}
    if world > 1:
        out["sample"] += "; the whole %d-rank job's workload, on rank 0 after the timed loop" % world
    return out


def workload_label(pm, S_total, H, smoothing, world, graph):
    """The BASELINE.json config a run's shape is (the prefix of config.workload), or "" for another
    shape.  configs[2] is 4096 x 64 per GPU (weak at N > 1), configs[3] 32768 x 64 in all,
    configs[4] 65536 x 128 with the Savitzky-Golay filter (window 10) and the captured graph."""
    if pm:
        return "BASELINE configs[1]: " if (S_total == 1024 and H == 32) else ""
    if S_total == 32768 and H == 64 and not smoothing:
        return "BASELINE configs[3]: "
    if S_total == 65536 and H == 128 and smoothing == 10:
        return "BASELINE configs[4]%s: " % ("" if graph == 1 else " (eager launches, not the hipGraph)")
    if S_total == 4096 * world and H == 64 and not smoothing:
        return "BASELINE configs[2]: " if world == 1 else "BASELINE configs[2]'s 4096 x 64 per GPU (weak): "
    return ""


def launch_ranks(n):
    """--gpus N > 1 without a launcher: start the N rank processes (this script again, one GPU
    each: LOCAL_RANK = RANK) with the rendezvous on 127.0.0.1, and return the exit status.  This
    process has imported no engine code and made no HIP call; it only waits.  If one rank fails
    the others are stopped (their exact PIDs), so a broken rendezvous does not hang the run."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 128 - rc


def rccl_check(infos, world):
    """Proof that the run was what it says: every rank's engine communicator reports `world` ranks
    (ncclCommCount) and its own rank (ncclCommUserRank), and the ranks sit on `world` distinct GPUs
    (PCI bus ids).  Returns the bench line's "rccl" entry; exits non-zero on any mismatch."""
    bad = []
    for i, x in enumerate(infos):
        if world > 1 and (x["nranks"] != world or x["rank"] != i):
            bad.append("rank %d: communicator reports %d ranks, rank %d" % (i, x["nranks"], x["rank"]))
    buses = [x["pci_bus_id"] for x in infos]
    if len(set(buses)) != len(buses):
        bad.append("ranks share a device: %s" % buses)
    if bad:
        sys.stderr.write("bench.py: RCCL check failed: %s\n" % "; ".join(bad))
        sys.exit(3)
    return {"ranks": world, "communicator_ranks": [x["nranks"] for x in infos],
            "devices": [{"rank": i, "hip_device": x["device"], "pci_bus_id": x["pci_bus_id"]} for i, x in enumerate(infos)]}


def bootstrap_only(world, rank, local_rank, dist):
    """MPPI_BENCH_BOOTSTRAP_ONLY=1 (CPU tests): stop after the gloo rendezvous and the broadcast of
    a stand-in for the RCCL unique id, before the engine loads; rank 0 prints what it saw.  The
    RCCL check runs on stand-ins for each rank's mppi_comm_info (MPPI_BENCH_STUB_NRANKS /
    MPPI_BENCH_STUB_SAME_DEVICE=1 make them wrong, to test the refusal)."""
    uid = [os.urandom(128) if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    stub_n = int(os.environ.get("MPPI_BENCH_STUB_NRANKS", world))
    same = os.environ.get("MPPI_BENCH_STUB_SAME_DEVICE") == "1"
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "local_rank": local_rank, "uid": uid[0].hex(), "pid": os.getpid(),
                                  "engine_loaded": "assistedmanipulation_amd" in sys.modules,
                                  "comm": {"nranks": stub_n, "rank": rank, "device": local_rank,
                                           "pci_bus_id": "0000:%02x:00.0" % (0 if same else local_rank)}})
    if rank == 0:
        rccl = rccl_check([x["comm"] for x in seen], world)
        print(json.dumps({"bootstrap_only": True, "n_gpus": world, "ranks": seen, "rccl": rccl}))
    dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (launch N ranks with --gpus N)" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # bootstrap + barrier / max-over-ranks only (gloo)
        dist.init_process_group("gloo")
        if os.environ.get("MPPI_BENCH_BOOTSTRAP_ONLY") == "1":
            bootstrap_only(world, rank, local_rank, dist)
            return
    run(args, world, rank, local_rank, dist)


def run(args, world, rank, local_rank, dist):
    global am, abi
    import assistedmanipulation_amd as am_  # the engine's ROCm runtime loads here, in the rank process
    from assistedmanipulation_amd import abi as abi_
    am, abi = am_, abi_
    create, unique_id = am.Trajectory.create, am.comm_unique_id
    if os.environ.get("MPPI_BENCH_STUB_ENGINE") == "1":   # CPU schema test: a stand-in engine (tests/bench_stub.py)
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import bench_stub
        create, unique_id = bench_stub.creator(world, rank), bench_stub.comm_unique_id
    pm = args.workload == "point_mass"
    S_total = args.samples_per_gpu * world
    horison = args.horizon_steps * 0.01
    sg = am.Smoothing(args.smoothing, 1) if (args.smoothing > 0 and not pm) else None
    if pm:
        conf = am.point_mass_configuration(rollouts=S_total, horison=horison, keep_best_rollouts=KEEP_BEST)
        traj = create(conf, am.PointMassDynamics(), am.QuadraticCost(), device=local_rank)
        default_workload = args.samples_per_gpu == 1024 and args.horizon_steps == 32
        x = np.zeros(6)
    else:
        conf = am.frankaridgeback_configuration(rollouts=S_total, horison=horison, keep_best_rollouts=KEEP_BEST,
                                                smoothing=sg)
        traj = create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation(), device=local_rank)
        # the shape the recorded PMC traffic was collected on (4096 x 64 per GPU, no filter)
        default_workload = args.samples_per_gpu == SAMPLES_PER_GPU and args.horizon_steps == 64 and sg is None
        x = am.huddled_state()
    if traj is None:
        raise SystemExit("engine create failed")
    comm1 = world == 1 and args.comm1 == 1
    if world > 1:
        uid = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        traj.comm_init(world, rank, uid[0])
        infos = [None] * world
        dist.all_gather_object(infos, traj.comm_info())
    else:
        if comm1:   # the sharded path on one GPU: a one-rank RCCL communicator
            traj.comm_init(1, 0, unique_id())
        try:
            infos = [traj.comm_info()]
        except AttributeError:   # an older library under an A/B run (MPPI_AMD_LIB) lacks mppi_comm_info
            infos = [{"nranks": 0, "rank": -1, "device": local_rank, "pci_bus_id": "unknown"}]
    rccl = rccl_check(infos, world)   # (every rank checks: a bad run stops before the timed loop)
    if comm1 and infos[0]["nranks"] != 1:
        sys.exit("bench.py: --comm1 but the engine reports %d communicator ranks" % infos[0]["nranks"])
    traj.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    if args.graph >= 0:
        traj.set_graph(args.graph)
    if not pm:
        traj.set_forecast(am.constant_forecast(traj.H))
    traj.set_timing(1)   # creates the engine's timing-event ring outside the timed region
    traj.set_timing(0)
    # HIP events around the rollout kernel on every EV_EVERY-th update of the timed region (each
    # event record delays the next kernel on the stream by ~4.5 us; the kernel's duration does not
    # vary, so a sample of the launches gives its average).  The engine keeps the event pairs and
    # they are read after the timed region (mppi_rollout_kernel_times).  The graph path replays only
    # updates without timing events, so with --graph 1 the timed loop records none and the rollout
    # launch is timed over EV_GRAPH further (eager) updates after it.
    sample_events = args.graph != 1
    j = 0
    for i in range(args.warmup):   # the timed loop's pattern (first event records happen here)
        sampled = sample_events and i % EV_EVERY == 0
        if sampled:
            traj.set_timing(1)
        traj.update(x, 0.05 * j)
        if sampled:
            traj.set_timing(0)
        j += 1
    if dist:
        dist.barrier()
    traj.rollout_kernel_times()    # clear the record
    g0 = traj.graph_updates()
    # the timed loop calls the C-ABI entry mppi_update itself (what a C++ caller of mppi_amd.hpp
    # calls), the constant state in the handle's buffer once, instead of Trajectory.update's
    # per-call copy and bookkeeping (≈0.7-1.3 us per update, tools/host_loop_probe.py)
    entry = traj.c_update_entry(x)   # (holds traj alive)
    upd, hnd, sptr = entry
    ok = abi.MPPI_OK
    t0 = time.perf_counter()
    for i in range(args.steps):
        sampled = sample_events and i % EV_EVERY == 0
        if sampled:
            traj.set_timing(1)
        st = upd(hnd, sptr, 0.05 * j)   # returns once U* is published; filter() overlaps the next update
        if st != ok:
            traj._check(st)
        if sampled:
            traj.set_timing(0)
        j += 1
    traj.synchronize()             # the last update's filter() finishes inside the timed region
    elapsed = time.perf_counter() - t0
    graph_timed = traj.graph_updates() - g0   # updates of the timed loop that ran as the hipGraph
    info = traj.update_info()      # what the engine's rollout launch did (its own choice, not re-derived)
    info["graph_updates_timed"] = graph_timed
    ev_source = "HIP events on every %d-th timed update" % EV_EVERY
    if not sample_events:   # the graph path: the rollout launch timed over further eager updates
        traj.set_timing(1)
        for _ in range(EV_GRAPH):
            traj.update(x, 0.05 * j)
            j += 1
        traj.set_timing(0)
        ev_source = "HIP events over %d eager updates after the timed (graph) loop" % EV_GRAPH
    dyn_times = traj.rollout_kernel_times()   # the rollout kernel's HIP-event times, sampled updates
    dyn_ms = sum(dyn_times) / max(len(dyn_times), 1)
    # the per-phase breakdown from a few further updates with every event recorded (untimed)
    traj.set_timing(2)
    kt = np.zeros(8)
    nb = 5
    for _ in range(nb):
        traj.update(x, 0.05 * j)
        kt += np.array(traj.kernel_times(detail=True))
        j += 1
    kt /= nb
    kt[3] = traj.kernel_times()[3]   # the optimal rollout (side stream) of the last update
    if dist:
        dist.barrier()
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    value = S_total * traj.H / (elapsed / args.steps)
    count_local = traj.R // world + (1 if rank < traj.R % world else 0)
    units = count_local * traj.H            # rollout-steps of this rank's rollout launch
    units_all = traj.R * traj.H             # of the whole update
    if pm:
        # the point mass is latency-bound, not HBM-bound: 0.8 MB of eps per update against a chain of
        # H dependent steps per rollout, one grid barrier and the publish (pm_update_kernel: the whole
        # update in one launch), or five dependent launches (MPPI_PM_FUSED=0).  The HBM view (the eps
        # written once and read once, fp64) is reported beside the latency, as the fraction of 8 TB/s
        # the launch's bytes reach.
        fused = bool(info.get("fused_update"))
        kernel = "pm_update_kernel (sample + rollouts + optimise + finish + filter + next rank/draws)" if fused \
            else "pm_rollout_kernel"
        rollout_bytes = 2 * 24.0 * units if fused else 24.0 * units
        roofline = {"bound": "latency", "kernel": kernel,
                    "critical_chain": "%d dependent rollout steps + a grid barrier + the publish, %s" % (
                        traj.H, "one launch per update" if fused else "five dependent launches per update"),
                    "achieved": rollout_bytes / (dyn_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "bytes_per_launch": rollout_bytes, "bytes_per_rollout_step": rollout_bytes / units,
                    "launch_us": dyn_ms * 1e3}
        roofline["frac"] = roofline["achieved"] / roofline["peak"]
        roofline["traffic"] = None
        if fused and os.path.exists(PMC_PM_JSON) and world == 1 and default_workload:
            with open(PMC_PM_JSON) as f:
                roofline["traffic"] = json.load(f)["traffic_bytes"]
            roofline["traffic_unit"] = "HBM bytes per launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)"
            roofline["traffic_source"] = recorded_label(PMC_PM_JSON)
        survey_bytes = BYTES_SURVEY_PM
    else:
        in_launch = info["objective_in_launch"] == 1
        flops_unit = FLOPS_PER_ROLLOUT_STEP if in_launch else FLOPS_DYN_PER_ROLLOUT_STEP
        rows_units = info["rows"] * traj.H   # rollout rows of the launch (+ a folded filter() row)
        achieved_tflops = flops_unit * rows_units / (dyn_ms * 1e-3) / 1e12
        traffic, traffic_note = None, None
        if os.path.exists(PMC_JSON) and default_workload and not comm1:
            with open(PMC_JSON) as f:
                traffic = json.load(f)["traffic_bytes"]
            if world > 1:   # rank 0's launch holds its 4096-4097 rollouts + the folded filter() row
                traffic_note = ("recorded for the N = 1 launch of 4099 rows; rank 0's launch here has %d rows"
                                % info["rows"])
        # the launch's HBM bytes by design: eps read, step records written and (objective in the
        # launch) read back, the next update's eps written in the tail (tail draws)
        launch_bytes = ((BYTES_EPS_FR + BYTES_REC * (2 if in_launch else 1)) * rows_units
                        + (BYTES_EPS_FR * units if info["tail_draws"] else 0.0))
        roofline = {"bound": "valu", "kernel": "fr_coop_x_kernel (dynamics + objective)" if in_launch else "fr_coop_kernel",
                    "compute": "fp64 VALU, issue-bound at one wave per SIMD (no dense contraction for MFMA)",
                    "achieved": achieved_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                    "traffic_unit": "HBM bytes per rollout launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)",
                    "traffic_source": recorded_label(PMC_JSON),
                    "flops_per_rollout_step": flops_unit,
                    "launch_bytes_by_design": launch_bytes,
                    "launch_GBs_by_design": launch_bytes / (dyn_ms * 1e-3) / 1e9,
                    "launch_time_source": ev_source}
        if traffic_note:
            roofline["traffic_note"] = traffic_note
        survey_bytes = BYTES_SURVEY_FR
    # SURVEY §8(d)'s algorithmic bytes per update (eps written once + read once by the reduce, fp64)
    # over the whole update's time: the HBM view of the metric; what the design moves beyond it (the
    # step records' round trip, the rollout's own eps read) is reported beside it as extra traffic
    hbm = {"survey_bytes_per_rollout_step": survey_bytes,
           "update_GBs_survey_bytes": survey_bytes * units_all / (ms_per_step * 1e-3) / 1e9,
           "peak_GBs": HBM_PEAK_GBS}
    hbm["frac_survey_bytes"] = hbm["update_GBs_survey_bytes"] / HBM_PEAK_GBS
    if not pm:
        hbm["extra_bytes_per_rollout_step"] = {"rollout_eps_read": BYTES_EPS_FR,
                                               "step_record_round_trip": 2 * BYTES_REC if info["objective_in_launch"] else BYTES_REC}
    # the weight reduce (weights_gradient_kernel): the HBM-bound kernel of the path - it reads the
    # [H][R][C] eps tensor once (96 B per rollout-step, fp64) and the costs; HIP events around it
    # alone in the untimed breakdown updates (kt[6]: behind the cost all-reduce when the engine's
    # RCCL communicator runs one, whose own time is kt[7]), PMC traffic from the profile set
    wg_ms = kt[6]
    if wg_ms > 0:
        wg_bytes = (BYTES_EPS_FR if not pm else 24.0) * units + 8.0 * traj.R   # the local eps, all R costs
        wg = {"kernel": "weights_gradient_kernel", "bound": "hbm",
              "ms": wg_ms, "bytes_per_launch": wg_bytes,
              "achieved_GBs": wg_bytes / (wg_ms * 1e-3) / 1e9, "peak_GBs": HBM_PEAK_GBS}
        wg["frac"] = wg["achieved_GBs"] / HBM_PEAK_GBS
        wg["traffic"] = None
        if world > 1 or comm1:
            wg["cost_allreduce_ms"] = kt[7]
            wg["note"] = "rank %d's shard; timed after the cost all-reduce (cost_allreduce_ms, RCCL), not including it" % rank
        if os.path.exists(PMC_WG_JSON) and world == 1 and not comm1 and default_workload and not pm:
            with open(PMC_WG_JSON) as f:
                rec = json.load(f)
            if wg["kernel"].split()[0] in rec["kernel"]:   # recorded for the kernel this run used
                wg["traffic"] = rec["traffic_bytes"]
                wg["traffic_source"] = recorded_label(PMC_WG_JSON)
        hbm["weight_reduce"] = wg
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    label = workload_label(pm, S_total, traj.H, args.smoothing if sg else 0, world, args.graph)
    if pm:
        workload = "%s%d samples x %d horizon, point-mass analytic dynamics + quadratic cost" % (label, S_total, traj.H)
        metric = "MPPI rollouts/sec (samples x horizon steps/s), %dx%d point mass" % (S_total, traj.H)
        data = "synthetic (x0 = 0, target (1,1,1), Philox noise)"
    else:
        workload = "%s%d samples x %d horizon, FrankaRidgeback Pinocchio dynamics, full AssistedManipulation cost stack%s%s%s" % (
            label, S_total, traj.H,
            ", Savitzky-Golay window %d order 1" % args.smoothing if sg else "",
            ", sample-sharded over RCCL" if world > 1 else (", through a one-rank RCCL communicator" if comm1 else ""),
            ", hipGraph-captured update" if args.graph == 1 else "")
        metric = "MPPI rollouts/sec (samples x horizon steps/s), %dx%d FrankaRidgeback" % (S_total, traj.H)
        data = "synthetic (HUDDLED state, constant forecast wrench (20,0,0) N, Philox noise)"
    line = {
        "metric": metric,
        "value": value,
        "unit": "rollout-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data,
        "config": {"workload": workload, "samples": S_total, "horizon": traj.H, "keep_best": KEEP_BEST,
                   "parallelism": "samples-dp%d" % world, "graph": args.graph, "comm1": int(comm1)},
        "engine": info,
        "kernel_ms": {"rollout_launch": dyn_ms, "rollout_launch_samples": len(dyn_times), "breakdown_untimed": {
                      "sample": kt[0], "rollout": kt[1], "reduce": kt[2], "weights_gradient": kt[6],
                      "cost_allreduce": kt[7], "optimal_rollout": kt[3], "update": kt[4]}},
        "roofline": roofline,
        "hbm": hbm,
        "rccl": rccl,
    }
    if not args.no_cpu_baseline:   # rank 0, after the timed loop: the whole job's workload
        line["cpu_baseline"] = cpu_baseline(args, pm, world)
        # not vs_baseline (no published number): the GPU / CPU-port ratio, same workload
        line["speedup_vs_cpu_baseline"] = value / line["cpu_baseline"]["value"]
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
