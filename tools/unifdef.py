"""Strip preprocessor conditionals on macros that are undefined for good (a small unifdef).

    python3 tools/unifdef.py FILE MACRO [MACRO ...]

Every `#ifdef M`, `#ifndef M`, `#if defined(M) ...` and `#elif defined(M)` whose condition only
names listed macros is resolved with those macros undefined, and the dead branch is deleted;
conditionals on anything else are kept as they are.  Rewrites FILE in place.
"""
import re
import sys


def evaluate(expr, macros):
    """True / False when `expr` names only listed macros (all undefined), else None."""
    names = re.findall(r"defined\s*\(\s*(\w+)\s*\)", expr)
    rest = re.sub(r"defined\s*\(\s*\w+\s*\)", "0", expr)
    if not names or any(n not in macros for n in names):
        return None
    if re.search(r"[A-Za-z_]", rest):
        return None
    return bool(eval(rest.replace("||", " or ").replace("&&", " and ").replace("!", " not ")))


def cond_of(line, macros):
    s = line.strip()
    m = re.match(r"#\s*ifdef\s+(\w+)", s)
    if m:
        return ("if", None if m.group(1) not in macros else False)
    m = re.match(r"#\s*ifndef\s+(\w+)", s)
    if m:
        return ("if", None if m.group(1) not in macros else True)
    m = re.match(r"#\s*if\s+(.*)", s)
    if m:
        return ("if", evaluate(m.group(1).split("//")[0], macros))
    m = re.match(r"#\s*elif\s+(.*)", s)
    if m:
        return ("elif", evaluate(m.group(1).split("//")[0], macros))
    if re.match(r"#\s*else\b", s):
        return ("else", None)
    if re.match(r"#\s*endif\b", s):
        return ("endif", None)
    return (None, None)


def process(lines, macros):
    out = []
    # stack entries: [resolved, keeping, taken]; resolved = this conditional is being removed
    stack = []

    def emitting():
        return all(e[1] for e in stack if e[0])

    for line in lines:
        kind, val = cond_of(line, macros)
        if kind == "if":
            if val is None:
                stack.append([False, True, False])
                if emitting():
                    out.append(line)
            else:
                stack.append([True, val, val])
            continue
        if kind in ("elif", "else", "endif") and stack:
            top = stack[-1]
            if top[0]:
                if kind == "endif":
                    stack.pop()
                elif kind == "else":
                    top[1] = not top[2]
                    top[2] = True
                else:
                    if val is None:
                        raise SystemExit("unresolvable #elif inside a resolved conditional: " + line)
                    top[1] = (not top[2]) and val
                    top[2] = top[2] or val
                continue
            if kind == "endif":
                stack.pop()
            if emitting():
                out.append(line)
            continue
        if emitting():
            out.append(line)
    if stack:
        raise SystemExit("unbalanced conditionals")
    return out


def main():
    path, macros = sys.argv[1], set(sys.argv[2:])
    with open(path) as f:
        lines = f.readlines()
    out = process(lines, macros)
    with open(path, "w") as f:
        f.writelines(out)
    print("%s: %d -> %d lines" % (path, len(lines), len(out)))


if __name__ == "__main__":
    main()
