"""Executed against algorithmic fp64 work per phase of the rollout step.

Executed: fr_coop.hip built to assembly with -DPHASE_MARKS (one comment per phase boundary, see the
PMARK macro); in the main step loop of fr_coop_x_kernel<1, false> (the four-wave update launch) every
instruction is attributed to the phase of the last marker before it, and fp64 VALU instructions count
2 FLOPs (v_fma_f64, v_fmac_f64, with or without DPP) or 1 (v_mul_f64, v_add_f64, v_rcp_f64) per
lane.  A wave carries four rollouts (16-lane rows), so executed FLOPs per rollout-step = per-lane
FLOPs x 64 / 4.  The objective runs in other waves, a lane per (rollout, step): its executed FLOPs per
rollout-step are one pass of fr_step_cost_kernel<1, false, false> (the same record_step_cost as the
launch's objective chunks) per lane, x 1.

Algorithmic: the oracle's FLOP-counting scalar over its minimal arithmetic (oracle_count_flops_phases:
zero-bias articulated-body solve, FK, kinematics, integration, get_cost), per rollout-step.  The
device's composite inertias + mass-matrix columns + Gauss-Jordan replace the oracle's solve.

usage: phase_flops.py [--asm FILE]   (default: compile assistedmanipulation_amd/csrc/fr_coop.hip and
fr_cost.hip with hipcc -DPHASE_MARKS into /tmp)
"""
import argparse
import collections
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "assistedmanipulation_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function", "-mllvm", "-disable-machine-licm",
         "-Wno-pass-failed", "--offload-device-only", "-S"]
DEV_PHASES = ["control + base velocity", "FK scan (+ sincos)", "world inertias", "kinematics for the cost",
              "composite inertias", "mass-matrix columns", "Gauss-Jordan solve", "integration + records"]
# device phase -> oracle phase (oracle.FLOP_PHASES)
DEV_TO_ALG = {0: "integration", 1: "fk", 2: "world_inertia", 3: "kinematics", 4: "solve", 5: "solve", 6: "solve",
              7: "integration"}


def flops_of(line):
    m = re.match(r"\s+(v_\w+)", line)
    if not m:
        return 0
    op = m.group(1)
    if re.match(r"v_(fma|fmac)_f64", op):
        return 2
    if re.match(r"v_(mul|add|rcp)_f64", op):
        return 1
    return 0


def compile_asm(src, out, extra=()):
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + FLAGS + list(extra) + [os.path.join(CSRC, src), "-o", out], cwd=CSRC)


def kernel_lines(path, symbol):
    lines, on = [], False
    for l in open(path):
        if l.startswith(symbol + ":"):
            on = True
            continue
        if on and l.startswith(".Lfunc_end"):
            break
        if on:
            lines.append(l)
    return lines


def step_loop(lines):
    """The self-looping basic block with the most instructions (the step loop)."""
    blocks, cur, lab = [], [], None
    for l in lines:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((lab, cur))
            lab, cur = m.group(1), []
            continue
        cur.append(l)
    blocks.append((lab, cur))
    loops = [(lab, b) for lab, b in blocks if lab and any(re.match(r"\s+s_cbranch_\w+\s+" + re.escape(lab) + r"\b", x) for x in b)]
    return max(loops, key=lambda x: sum(1 for y in x[1] if re.match(r"\s+[vsdg]\w+_", y)))


def device_phases(asm):
    sym = [l.split(":")[0] for l in open(asm) if re.match(r"^_Z16fr_coop_x_kernelILi1ELb0EE\S*:", l)][0]
    lab, body = step_loop(kernel_lines(asm, sym))
    # the loop block starts in the phase its back edge left (the last marker of the block)
    marks = [int(m.group(1)) for m in (re.search(r"; PHASE (\d)", l) for l in body) if m]
    ph = marks[-1] if marks else 0
    inst, fl = collections.Counter(), collections.Counter()
    for l in body:
        m = re.search(r"; PHASE (\d)", l)
        if m:
            ph = int(m.group(1))
            continue
        if re.match(r"\s+(v_|s_|ds_|global_|buffer_)", l):
            inst[ph] += 1
            fl[ph] += flops_of(l)
    return lab, inst, fl


def objective_flops(asm):
    sym = [l.split(":")[0] for l in open(asm) if re.match(r"^_Z\S*fr_step_cost_kernelILi1ELb0ELb0EE\S*:", l)][0]
    body = kernel_lines(asm, sym)
    # one pass (H <= 64): the straight-line body; the per-joint parameter staging loop and the
    # readlane sum are outside the step cost (counted anyway: a small upper bound)
    return sum(flops_of(l) for l in body), sum(1 for l in body if re.match(r"\s+(v_|s_|ds_|global_)", l))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--asm", default="/tmp/phase_fr_coop.s")
    p.add_argument("--cost-asm", default="/tmp/phase_fr_cost.s")
    p.add_argument("--no-build", action="store_true")
    a = p.parse_args()
    if not a.no_build:
        compile_asm("fr_coop.hip", a.asm, ["-DPHASE_MARKS"])
        compile_asm("fr_cost.hip", a.cost_asm)
    sys.path.insert(0, REPO)
    import assistedmanipulation_amd as am
    from oracle import oracle as O
    tot, alg = O.count_flops_phases(am.FrankaRidgebackDynamics().descriptor().frankaridgeback,
                                    am.AssistedManipulation().descriptor().assisted_manipulation, am.huddled_state())
    lab, inst, fl = device_phases(a.asm)
    obj_fl, obj_inst = objective_flops(a.cost_asm)
    print("step loop %s of fr_coop_x_kernel<1, false> (PHASE_MARKS build): %d instructions" % (lab, sum(inst.values())))
    print("%-26s %6s %10s %12s %12s %7s" % ("phase", "instr", "FLOP/lane", "exec/r-step", "alg/r-step", "ratio"))
    grouped = collections.OrderedDict()
    for d in range(8):
        ex = fl[d] * 64 / 4
        print("%-26s %6d %10d %12.0f %12s %7s" % (DEV_PHASES[d], inst[d], fl[d], ex, "", ""))
        g = DEV_TO_ALG[d]
        grouped[g] = grouped.get(g, 0.0) + ex
    grouped["objective"] = float(obj_fl)
    print("%-26s %6d %10d %12.0f %12s %7s" % ("objective (other waves)", obj_inst, obj_fl, obj_fl, "", ""))
    print()
    print("%-16s %12s %12s %7s" % ("oracle phase", "exec/r-step", "alg/r-step", "ratio"))
    te = 0.0
    for g in O.FLOP_PHASES:
        ex = grouped.get(g, 0.0)
        te += ex
        print("%-16s %12.0f %12.0f %7.2f" % (g, ex, alg[g], ex / alg[g] if alg[g] else float("nan")))
    print("%-16s %12.0f %12.0f %7.2f" % ("total", te, tot, te / tot))


if __name__ == "__main__":
    main()
