"""Resolve preprocessor switches with known values out of a source file.

    python tools/unifdef.py FILE -D NAME=VALUE ... -U NAME ...

Every #if / #ifdef / #ifndef / #elif / #else / #endif whose condition uses only
the named macros is evaluated and removed (the taken branch kept); conditions
that involve any other macro are left as they are.  The file is rewritten in
place; remaining uses of the resolved names in code lines are listed on stderr
(they need a constant in their place).
"""
import argparse
import re
import sys

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")


def evaluate(expr, known):
    """-> bool, or None when the expression uses an unknown macro."""
    expr = re.sub(r"//.*$", "", expr)
    expr = re.sub(r"/\*.*?\*/", "", expr)

    def defined(m):
        name = m.group(1)
        if name not in known:
            raise KeyError(name)
        return "1" if known[name] is not None else "0"

    try:
        expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)", defined, expr)
        expr = re.sub(r"defined\s+(\w+)", defined, expr)

        def ident(m):
            name = m.group(0)
            if name not in known:
                raise KeyError(name)
            v = known[name]
            return "0" if v is None else str(v)

        expr = re.sub(r"\b[A-Za-z_]\w*\b", ident, expr)
    except KeyError:
        return None
    expr = expr.replace("&&", " and ").replace("||", " or ")
    expr = re.sub(r"!(?!=)", " not ", expr)
    return bool(eval(expr, {}, {}))


def process(lines, known):
    out = []
    stack = []  # frames: dict(resolved, taking, taken, parent_live)

    def live():
        return all(f["taking"] for f in stack if f["resolved"])

    for line in lines:
        m = DIRECTIVE.match(line)
        if not m:
            if live():
                out.append(line)
            continue
        kind, rest = m.group(1), m.group(2).strip()
        if kind in ("if", "ifdef", "ifndef"):
            if kind == "if":
                v = evaluate(rest, known)
            else:
                name = rest.split()[0]
                v = None if name not in known else ((known[name] is not None) == (kind == "ifdef"))
            if v is None:
                stack.append({"resolved": False})
                if live():
                    out.append(line)
            else:
                stack.append({"resolved": True, "taking": v, "taken": v})
        elif kind == "elif":
            f = stack[-1]
            if not f["resolved"]:
                if live():
                    out.append(line)
                continue
            if f["taken"]:
                f["taking"] = False
            else:
                v = evaluate(rest, known)
                if v is None:
                    raise SystemExit(f"unresolvable #elif after a resolved #if: {line.strip()}")
                f["taking"] = f["taken"] = v
        elif kind == "else":
            f = stack[-1]
            if not f["resolved"]:
                if live():
                    out.append(line)
                continue
            f["taking"] = not f["taken"]
            f["taken"] = True
        else:  # endif
            f = stack.pop()
            if not f["resolved"] and live():
                out.append(line)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("file")
    p.add_argument("-D", action="append", default=[])
    p.add_argument("-U", action="append", default=[])
    a = p.parse_args()
    known = {}
    for d in a.D:
        k, _, v = d.partition("=")
        known[k] = v or "1"
    for u in a.U:
        known[u] = None
    src = open(a.file).read().split("\n")
    out = process(src, known)
    open(a.file, "w").write("\n".join(out))
    for i, line in enumerate(out, 1):
        if DIRECTIVE.match(line):
            continue
        for name in known:
            if re.search(r"\b%s\b" % re.escape(name), line):
                print(f"{a.file}:{i}: {name} still used: {line.strip()}", file=sys.stderr)


if __name__ == "__main__":
    main()
