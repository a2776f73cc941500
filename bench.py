#!/usr/bin/env python3
"""MPPI rollout throughput on MI355X — BASELINE.json's metric.

A "step" is one mppi::Trajectory::update() (reference src/controller/mppi.cpp:154-187, its own
timing boundary) of the FrankaRidgeback Pinocchio dynamics + full AssistedManipulation cost,
4096 samples x 64-step horizon per GPU (BASELINE configs[2]; configs[3] at N = 8), with the
reference's cadence: updates at t = 0.05 j (5-step shift), keep-best 20, device Philox noise.
value = samples x horizon x ranks / (max-over-ranks seconds per update).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import assistedmanipulation_amd as am  # noqa: E402  (engine's ROCm runtime loads first)
from assistedmanipulation_amd import abi  # noqa: E402

SAMPLES_PER_GPU = 4096
HORISON = 0.64            # 64 steps at dt = 0.01
KEEP_BEST = 20
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 vector (= fp64 matrix) peak, AMD spec; the rollout is fp64 VALU
# Algorithmic FLOPs of one rollout-step of the minimal arithmetic the device executes
# (world-frame zero-bias ABA + kinematics + default cost), counted by the oracle's
# FLOP-counting scalar (tests/test_oracle_cpu.py::test_flop_count_constant pins these values):
# the cost part (get_cost) runs in fr_step_cost_kernel, the rest in the rollout kernel.
FLOPS_PER_ROLLOUT_STEP = 6518.0
FLOPS_COST_PER_ROLLOUT_STEP = 690.0
FLOPS_DYN_PER_ROLLOUT_STEP = FLOPS_PER_ROLLOUT_STEP - FLOPS_COST_PER_ROLLOUT_STEP
# Algorithmic HBM bytes per rollout-step: the rollout launch reads its eps column (C = 12 fp64)
# once; on the records path it also writes a step record (FR_NREC = 42 fp64) the cost kernel reads.
BYTES_EPS_PER_ROLLOUT_STEP = 96.0
BYTES_REC_PER_ROLLOUT_STEP = 336.0
BYTES_PER_ROLLOUT_STEP = BYTES_EPS_PER_ROLLOUT_STEP + BYTES_REC_PER_ROLLOUT_STEP
# HBM traffic per rollout launch measured by rocprofv3 PMC passes (tools/gpu_pmc.sh ->
# tools/pmc_traffic.py): FETCH_SIZE (x2, gfx950) + WRITE_SIZE of the main rollout dispatch.
EV_EVERY = 8   # timed updates per rollout-kernel event sample
PMC_JSON = os.path.join(HERE, "profiles", "r02_pmc_rollout.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 200 timed updates (~60 ms): the last update's filter(), finished inside the timed region by
    # the closing synchronize (~0.18 ms alone), is spread over the steady-state updates
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--samples-per-gpu", type=int, default=SAMPLES_PER_GPU)
    p.add_argument("--horizon-steps", type=int, default=int(round(HORISON / 0.01)),
                   help="H (dt = 0.01); 64 = configs[2]/[3], 128 = configs[4]")
    p.add_argument("--smoothing", type=int, default=0,
                   help="Savitzky-Golay window (order 1); 10 = configs[4]")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16)
    return p.parse_args()


def cpu_baseline(threads, samples, horison):
    """The oracle (fp64 restatement of the reference's CPU mppi.cpp path, Pinocchio-order
    arithmetic, contiguous-block thread partition of mppi.cpp:272-307) on this host: a bounded
    sample of the same workload (a few full updates)."""
    from oracle import oracle as O
    try:
        libpath = O.build(native=True)   # g++ -O3 -march=native on the GPU box host
    except Exception:
        libpath = O.LIB_PATH
    conf = am.frankaridgeback_configuration(rollouts=samples, horison=horison, keep_best_rollouts=KEEP_BEST,
                                            threads=threads)
    cc, keep = conf.to_c()
    orc = O.OracleTrajectory(cc, am.FrankaRidgebackDynamics().descriptor(), am.AssistedManipulation().descriptor(),
                             lib_path=libpath)
    orc.set_noise_source(False, 12345)
    orc.set_forecast(am.constant_forecast(orc.H))
    x = am.huddled_state()
    orc.update(x, 0.0)   # warm-up
    durs = []
    t_total = 0.0
    j = 1
    while j <= 8 and (t_total < 10.0 or j <= 2):
        orc.update(x, 0.05 * j)
        d = orc.update_duration()
        durs.append(d)
        t_total += d
        j += 1
    med = float(np.median(durs))
    return {"value": samples * orc.H / med, "unit": "rollout-steps/s", "cores": threads, "kind": "port",
            "sample": "%d timed updates of the %dx%d FrankaRidgeback workload (median %.3f s/update), "
                      "oracle/mppi_oracle.cpp fp64, %d threads, -march=native" % (len(durs), samples, orc.H, med, threads)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # bootstrap + barrier / max-over-ranks only (gloo)
        dist.init_process_group("gloo")
    S_total = args.samples_per_gpu * world
    horison = args.horizon_steps * 0.01
    sg = am.Smoothing(args.smoothing, 1) if args.smoothing > 0 else None
    default_workload = args.samples_per_gpu == SAMPLES_PER_GPU and args.horizon_steps == 64 and sg is None
    conf = am.frankaridgeback_configuration(rollouts=S_total, horison=horison, keep_best_rollouts=KEEP_BEST,
                                            smoothing=sg)
    traj = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation(), device=local_rank)
    if traj is None:
        raise SystemExit("engine create failed")
    if world > 1:
        uid = [am.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        traj.comm_init(world, rank, uid[0])
    traj.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    traj.set_forecast(am.constant_forecast(traj.H))
    x = am.huddled_state()
    traj.set_timing(1)   # creates the engine's timing-event ring outside the timed region
    traj.set_timing(0)
    j = 0
    for i in range(args.warmup):   # the timed loop's pattern (first event records happen here)
        sampled = i % EV_EVERY == 0
        if sampled:
            traj.set_timing(1)
        traj.update(x, 0.05 * j)
        if sampled:
            traj.set_timing(0)
        j += 1
    if dist:
        dist.barrier()
    # HIP events around the rollout kernel on every EV_EVERY-th update of the timed region (each
    # event record delays the next kernel on the stream by ~4.5 us; the kernel's duration does not
    # vary, so a sample of the launches gives its average).  The engine keeps the event pairs and
    # they are read after the timed region (mppi_rollout_kernel_times).
    traj.rollout_kernel_times()    # clear the record
    t0 = time.perf_counter()
    for i in range(args.steps):
        sampled = i % EV_EVERY == 0
        if sampled:
            traj.set_timing(1)
        traj.update(x, 0.05 * j)   # returns once U* is published; filter() overlaps the next update
        if sampled:
            traj.set_timing(0)
        j += 1
    traj.synchronize()             # the last update's filter() finishes inside the timed region
    elapsed = time.perf_counter() - t0
    dyn_times = traj.rollout_kernel_times()   # the rollout kernel's HIP-event times, sampled updates
    dyn, nd = sum(dyn_times), len(dyn_times)
    # the per-phase breakdown from a few further updates with every event recorded (untimed)
    traj.set_timing(2)
    kt = np.zeros(6)
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
    lane = os.environ.get("MPPI_FR_KERNEL") == "lane"   # A/B: the fused one-lane-per-rollout kernel
    dyn_ms = dyn / max(nd, 1)                             # the rollout (dynamics) kernel alone, timed loop
    records = not lane   # the coop kernel writes step records; the objective reads them back
    # one round of four-wave workgroups (fr_coop.hip fr_coop_update_fusable): the launch evaluates
    # the objective itself in the SIMDs' idle tail (MPPI_COSTS_IN_LAUNCH=0: fr_step_cost_kernel)
    count_all = traj.R // world + (1 if rank < traj.R % world else 0)
    groups = count_all // 16
    xrows = count_all - 16 * groups + (1 if count_all - 16 * groups > 0 else 0)
    in_launch = records and os.environ.get("MPPI_COSTS_IN_LAUNCH") != "0" and 0 < groups <= 256 and xrows <= 4 * groups
    # the launch's tail also writes the next update's eps of its main waves' rows (tail_draws)
    tail_draws = in_launch and xrows > 0 and os.environ.get("MPPI_TAIL_DRAWS") != "0" and os.environ.get("MPPI_DRAW_AHEAD") != "0"
    cost_ms = float(kt[1] - kt[5]) if records and not in_launch else 0.0   # fr_step_cost_kernel (breakdown pass)
    traffic = None
    if os.path.exists(PMC_JSON) and world == 1 and default_workload:
        with open(PMC_JSON) as f:
            traffic = json.load(f)["traffic_bytes"]
    count_local = traj.R // world + (1 if rank < traj.R % world else 0)
    units = count_local * traj.H
    flops_unit = FLOPS_DYN_PER_ROLLOUT_STEP if records and not in_launch else FLOPS_PER_ROLLOUT_STEP
    flops = flops_unit * units
    achieved_tflops = flops / (dyn_ms * 1e-3) / 1e12
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    line = {
        "metric": "MPPI rollouts/sec (samples x horizon steps/s), %dx%d FrankaRidgeback" % (S_total, traj.H),
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
        "data": "synthetic (HUDDLED state, constant forecast wrench (20,0,0) N, Philox noise)",
        "config": {"workload": "%s%d samples x %d horizon, FrankaRidgeback Pinocchio dynamics, "
                               "full AssistedManipulation cost stack%s%s" % (
                                   ("BASELINE configs[%d]: " % (2 if world == 1 else 3)) if default_workload else "",
                                   S_total, traj.H, ", Savitzky-Golay window %d order 1" % args.smoothing if sg else "",
                                   ", sample-sharded over RCCL" if world > 1 else ""),
                   "samples": S_total, "horizon": traj.H, "keep_best": KEEP_BEST, "parallelism": "samples-dp%d" % world},
        "kernel_ms": {"rollout_dynamics": dyn_ms, "rollout_cost": cost_ms, "breakdown_untimed": {
                      "sample": kt[0], "rollout": kt[1], "reduce": kt[2], "optimal_rollout": kt[3], "update": kt[4]}},
        # The rollout kernel runs fp64 VALU work (no MFMA: the 12-body chain has no dense contraction)
        # at one wave per SIMD, so it is bound by issue slots and dependency chains, not by a
        # datapath peak; the fraction is reported against the fp64 vector peak.
        "roofline": {"bound": "valu", "compute": "fp64 VALU, latency/issue-bound at one wave per SIMD",
                     "kernel": "fr_rollout_kernel" if lane else ("fr_coop_x_kernel (dynamics + objective)" if in_launch else "fr_coop_x_kernel"),
                     "achieved": achieved_tflops,
                     "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved_tflops / FP64_PEAK_TFLOPS,
                     "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, %s)" % os.path.relpath(PMC_JSON, HERE),
                     "flops_per_rollout_step": flops_unit},
        "hbm": {"rollout_algorithmic_GBs": ((BYTES_PER_ROLLOUT_STEP + (BYTES_REC_PER_ROLLOUT_STEP if in_launch else 0.0)
                                             + (BYTES_EPS_PER_ROLLOUT_STEP if tail_draws else 0.0))
                                            if records else BYTES_EPS_PER_ROLLOUT_STEP) * units / (dyn_ms * 1e-3) / 1e9,
                "objective_in_rollout_launch": in_launch,
                "cost_kernel_algorithmic_GBs": BYTES_REC_PER_ROLLOUT_STEP * units / (cost_ms * 1e-3) / 1e9 if records and cost_ms > 0 else None,
                "peak_GBs": HBM_PEAK_GBS},
    }
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_threads, args.samples_per_gpu, horison)
        # not vs_baseline (no published number): the GPU / CPU-port ratio, same workload
        line["speedup_vs_cpu_baseline"] = value / line["cpu_baseline"]["value"]
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
