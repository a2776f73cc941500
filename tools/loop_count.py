"""Instructions per horizon step of the cooperative rollout kernels: the step is one basic block
 that branches back to itself, so the self-loop blocks of a kernel with more than 200
instructions in the device assembly (fr_coop.s, written by the Makefile) are its step loops (one
per coop_rows copy: main rows, relay).  usage: loop_count.py file.s [symbol-substring ...]"""
import re
import sys


def blocks(path):
    """{kernel symbol: [(label, instruction count, {kind: count}, branches back to itself)]}"""
    out, cur, lab, n, kinds, selfloop = {}, None, None, 0, {}, False
    for line in open(path):
        if re.match(r"^_Z\S+:\s*(;.*)?$", line) or re.match(r"^[A-Za-z_]\w*:\s*(;.*)?$", line) and not line.startswith("."):
            if cur is not None and lab is not None:
                out[cur].append((lab, n, kinds, selfloop))
            cur = line.split(":")[0]
            out.setdefault(cur, [])
            lab, n, kinds, selfloop = "entry", 0, {}, False
            continue
        if cur is None:
            continue
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            out[cur].append((lab, n, kinds, selfloop))
            lab, n, kinds, selfloop = m.group(1), 0, {}, False
            continue
        if line.startswith(".Lfunc_end"):
            out[cur].append((lab, n, kinds, selfloop))
            cur, lab = None, None
            continue
        b = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", line)
        if b and b.group(1) == lab:
            selfloop = True
        m = re.match(r"\s+(v_|ds_|s_|global_|buffer_|scratch_)(\S*)", line)
        if m:
            n += 1
            w = m.group(1) + m.group(2)
            k = w if w in ("s_nop", "s_waitcnt") else m.group(1) + ("dpp" if "dpp" in line or "row_" in line else "")
            kinds[k] = kinds.get(k, 0) + 1
    return out


def main(path, subs):
    for sym, bl in blocks(path).items():
        if subs and not any(s in sym for s in subs):
            continue
        if not bl:
            continue
        loops = [b for b in bl if b[3] and b[1] > 200]
        for lab, n, kinds, _ in loops:
            print("%-70s step loop %s: %d instructions %s" % (sym[:70], lab, n, kinds))
        if not loops:
            lab, n, kinds, _ = max(bl, key=lambda b: b[1])
            print("%-70s largest block %s: %d instructions %s" % (sym[:70], lab, n, kinds))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
