"""Check the gfx9 DPP read-after-VALU-write hazard in a kernel's ISA: a DPP instruction may not read
(as its DPP source, src0) a VGPR that a VALU instruction wrote fewer than two wait states before
(instructions in between, or s_nop N = N + 1).  The rollout kernel's hand-written DPP blocks drop the
defensive s_nop where the generated order already leaves the distance; this verifies it on the
compiled code (straight-line: the horizon loop is one basic block).

usage: dpp_hazard_check.py file.s [kernel_symbol_prefix]   (default: every kernel in the file)"""
import re
import sys


def regs(tok):
    """VGPR numbers named by an operand token (v5, v[4:5])."""
    tok = tok.strip().lstrip("-|").rstrip("|")
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def check(path, prefix="", strict=True):
    bad = 0
    inside = False
    recent, trans = [], []
    in_asm, since_label = False, 2   # (wait states since the write, registers)
    for l in open(path):
        l = l.rstrip("\n")
        if not inside:
            m = re.match(r"^(_Z\w+):", l)
            if m and m.group(1).startswith(prefix or "_Z"):
                inside, recent, trans = True, [], []
            continue
        if l.startswith(".Lfunc_end"):
            inside = False
            continue
        s = l.strip()
        if s == ";;#ASMSTART":
            in_asm = True
        elif s == ";;#ASMEND":
            in_asm = False
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            if s.endswith(":"):
                recent, trans = [], []   # a branch target: the distance is only tracked in straight-line code
                since_label = 0
            continue
        op = s.split()[0]
        ws = int(s.split()[1], 0) + 1 if op == "s_nop" else 1
        # hand-written DPP within two wait states of a branch target: the writes before the label
        # are not seen here (and LLVM cannot pad inside inline asm), so the distance is unverified
        if in_asm and since_label < 2 and ("_dpp" in op or " row_" in s):
            print("unverified (asm DPP at a block start): %s" % s)
            bad += 1
        since_label += ws
        if "_dpp" in op or " row_" in s or "quad_perm" in s:
            ops = s[len(op):].split(",")
            src0 = regs(ops[1]) if len(ops) > 1 else set()
            # the other sources too, as LLVM's hazard recognizer counts them (conservative: the
            # documented hazard is the operand read through the DPP network, src0)
            srcs = set().union(*[regs(o.split()[0]) for o in ops[1:] if o.strip()]) if len(ops) > 1 else set()
            for dist, w in recent:
                if dist < 2 and (w & src0):
                    print("hazard (%d wait states): %s" % (dist, s))
                    bad += 1
                elif dist < 2 and (w & srcs) and strict:
                    print("hazard on a non-DPP source (%d wait states): %s" % (dist, s))
                    bad += 1
        # gfx940+ trans forwarding: a VALU reading a transcendental's result (v_rcp / v_rsq / v_sqrt /
        # v_exp / v_log / v_sin / v_cos) in the very next instruction reads a stale value
        if op.startswith("v_") and "_dpp" not in op:
            srcs = set().union(*[regs(o.split()[0]) for o in s[len(op):].split(",")[1:] if o.strip()]) \
                if "," in s else set()
            for dist, w in trans:
                if dist < 1 and (w & srcs):
                    print("trans forwarding hazard: %s" % s)
                    bad += 1
        recent = [(d + ws, w) for d, w in recent if d + ws < 2]
        trans = [(d + ws, w) for d, w in trans if d + ws < 1]
        if op.startswith("v_") and op != "v_nop":
            dst = regs(s[len(op):].split(",")[0])
            if dst:
                recent.append((0, dst))
                if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", op):
                    trans.append((0, dst))
    return bad


if __name__ == "__main__":
    n = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    print("dpp_hazard_check: %d DPP read-after-write hazards in %s" % (n, sys.argv[1]))
    sys.exit(1 if n else 0)
