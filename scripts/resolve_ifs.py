#!/usr/bin/env python3
"""Resolve preprocessor conditionals on chosen macros in place (a tiny unifdef).

    python scripts/resolve_ifs.py FILE NAME=VALUE ...   (VALUE "undef" = not defined)

Only #if/#ifdef/#ifndef/#elif lines whose expression names nothing but the given
macros (plus integer literals, ! && || == != < > <= >= and parentheses) are
resolved; every other conditional is kept verbatim (its nesting is tracked).
The `#ifndef M / #define M v / #endif` default blocks of resolved macros go too.
Used to prune recorded-negative A/B switches (profiles/ keeps their record).
"""
import re
import sys


def main():
    path = sys.argv[1]
    vals = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        vals[k] = None if v == "undef" else int(v, 0)
    lines = open(path).read().split("\n")
    out = []
    # stack entries: (resolved?, emitting?, any_branch_taken?, parent_emitting)
    stack = []

    def emitting():
        return all(e[1] for e in stack)

    def evaluate(expr):
        toks = re.findall(r"[A-Za-z_]\w*|\d+|&&|\|\||==|!=|<=|>=|[!<>()]", expr)
        py = []
        for t in toks:
            if t == "defined":
                py.append("_defined")
                continue
            if re.match(r"[A-Za-z_]", t):
                if t not in vals:
                    return None
                py.append(f"_v('{t}')")
            elif t == "&&":
                py.append(" and ")
            elif t == "||":
                py.append(" or ")
            elif t == "!":
                py.append(" not ")
            else:
                py.append(t)
        src = "".join(py)
        src = re.sub(r"_defined\s*\(\s*_v\('(\w+)'\)\s*\)", r"_d('\1')", src)
        src = re.sub(r"_defined\s*_v\('(\w+)'\)", r"_d('\1')", src)
        return bool(eval(src, {"_v": lambda k: vals[k] or 0, "_d": lambda k: vals[k] is not None}))

    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", ln)
        if not m:
            if emitting():
                out.append(ln)
            i += 1
            continue
        kw, rest = m.group(1), re.sub(r"//.*|/\*.*?\*/", "", m.group(2)).strip()
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "if":
                r = evaluate(rest)
            else:
                name = rest.split()[0]
                if name in vals:
                    d = vals[name] is not None
                    r = d if kw == "ifdef" else not d
                    # default block `#ifndef M / #define M v / #endif`: drop it
                    if kw == "ifndef" and i + 2 < len(lines) and re.match(rf"\s*#\s*define\s+{name}\b", lines[i + 1]) \
                            and re.match(r"\s*#\s*endif", lines[i + 2]):
                        i += 3
                        continue
                else:
                    r = None
            if r is None:
                stack.append((False, True, True))
                if emitting():
                    out.append(ln)
            else:
                stack.append((True, r, r))
        elif kw == "elif":
            res, emit, taken = stack[-1]
            if not res:
                stack[-1] = (res, emit, taken)
                if emitting():
                    out.append(ln)
            else:
                r = evaluate(rest)
                if r is None:
                    raise SystemExit(f"{path}:{i + 1}: #elif on an unknown macro after a resolved #if")
                stack[-1] = (True, (not taken) and r, taken or r)
        elif kw == "else":
            res, emit, taken = stack[-1]
            if not res:
                if emitting():
                    out.append(ln)
            else:
                stack[-1] = (True, not taken, True)
        else:  # endif
            res, _, _ = stack.pop()
            if not res and emitting():
                out.append(ln)
        i += 1
    if stack:
        raise SystemExit(f"{path}: unbalanced conditionals")
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
