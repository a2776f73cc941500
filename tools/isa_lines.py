"""Attribute the VALU/LDS/SALU instructions of one kernel in a -save-temps .s file (built with
-gline-tables-only) to source lines.  usage: isa_lines.py file.s kernel_symbol_prefix [top]"""
import collections
import re
import sys


def main(path, sym, top=40):
    files, cnt, kinds = {}, collections.Counter(), collections.Counter()
    cur, inside = None, False
    for line in open(path):
        if line.startswith(sym):
            inside = True
            continue
        if inside and line.startswith(".Lfunc_end"):
            break
        m = re.match(r'\s+\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if not inside:
            continue
        m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        m = re.match(r"\s+(v_|ds_|s_|global_|buffer_|scratch_)(\S*)", line)
        if m:
            cnt[cur] += 1
            kinds[m.group(1)] += 1
    print("total", sum(cnt.values()), dict(kinds))
    srcs = {}
    for (f, ln), c in sorted(cnt.items(), key=lambda x: -x[1])[:top]:
        name = files.get(f, f)
        txt = ""
        if name.endswith(".hip") or name.endswith(".hpp"):
            for d in ("assistedmanipulation_amd/csrc/",):
                try:
                    srcs.setdefault(name, open(d + name).read().split("\n"))
                    txt = srcs[name][ln - 1].strip()[:90]
                except OSError:
                    pass
        print("%5d %s:%d  %s" % (c, name, ln, txt))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
