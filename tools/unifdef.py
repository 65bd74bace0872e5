"""Resolve preprocessor conditionals on known macro values (a small unifdef):
python tools/unifdef.py -DNAME=VAL ... file [file ...] rewrites the files in
place. A condition is resolved only when every identifier in it is known
(defined(X) included); other conditionals are kept as they are. `#ifndef X /
#define X v / #endif` default blocks of a resolved macro are dropped."""
import re
import sys


def parse_args(argv):
    vals, files = {}, []
    for a in argv:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            vals[k] = int(v or "1")
        else:
            files.append(a)
    return vals, files


def evaluate(expr, vals):
    expr = re.sub(r"//.*$", "", expr)
    expr = re.sub(r"/\*.*?\*/", "", expr).strip()
    ids = set(re.findall(r"[A-Za-z_]\w*", expr)) - {"defined"}
    if not ids <= set(vals):
        return None
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1", expr)
    e = re.sub(r"defined\s+(\w+)", lambda m: "1", e)
    e = re.sub(r"[A-Za-z_]\w*", lambda m: str(vals[m.group(0)]), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    return bool(eval(e))


def process(lines, vals):
    out = []
    # stack entries: (mode, taken) ; mode 'keep' = directive kept verbatim,
    # 'res' = resolved (emit branch contents only when active)
    stack = []
    active = lambda: all(s["emit"] for s in stack)
    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)$", ln)
        if not m:
            if active():
                out.append(ln)
            i += 1
            continue
        d, rest = m.group(1), m.group(2).strip()
        if d in ("if", "ifdef", "ifndef"):
            name = rest.split()[0] if rest else ""
            if d == "ifdef":
                c = True if name in vals else None
            elif d == "ifndef":
                c = False if name in vals else None
            else:
                c = evaluate(rest, vals)
            if c is None:
                stack.append(dict(res=False, emit=True, taken=False))
                if active():
                    out.append(ln)
            else:
                stack.append(dict(res=True, emit=c, taken=c))
        elif d == "elif":
            s = stack[-1]
            if not s["res"]:
                c = evaluate(rest, vals)
                if c is None:
                    if all(x["emit"] for x in stack[:-1]):
                        out.append(ln)
                else:
                    # a resolved #elif in a kept chain: emit as #elif 1/0 for simplicity
                    if all(x["emit"] for x in stack[:-1]):
                        out.append(re.sub(r"#\s*elif.*", "#elif %d" % int(c), ln))
            else:
                c = evaluate(rest, vals)
                if c is None:
                    raise SystemExit("unresolvable #elif after a resolved #if: %r" % ln)
                s["emit"] = (not s["taken"]) and c
                s["taken"] = s["taken"] or c
        elif d == "else":
            s = stack[-1]
            if s["res"]:
                s["emit"] = not s["taken"]
                s["taken"] = True
            elif all(x["emit"] for x in stack[:-1]):
                out.append(ln)
        else:  # endif
            s = stack.pop()
            if not s["res"] and active():
                out.append(ln)
        i += 1
    assert not stack, "unbalanced conditionals"
    return out


def main():
    vals, files = parse_args(sys.argv[1:])
    for f in files:
        src = open(f).read().split("\n")
        res = process(src, vals)
        # drop '#define NAME value' lines of resolved macros
        res = [l for l in res if not any(re.match(r"\s*#\s*define\s+%s\b" % k, l) for k in vals)]
        open(f, "w").write("\n".join(res))


if __name__ == "__main__":
    main()
