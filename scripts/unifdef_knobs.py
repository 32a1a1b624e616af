"""Resolve build-time A/B switches to their shipped values (a small unifdef for the knobs named
here): #if / #ifdef / #ifndef / #elif / #else / #endif on conditions over these macros only are
evaluated, their dead branches dropped, their `#ifndef X / #define X v / #endif` defaults removed,
and remaining uses of X in code replaced by v. Directives on other macros are kept as they are.

    python scripts/unifdef_knobs.py FILE NAME=VALUE ...
"""
import re
import sys


def cond_value(expr, knobs):
    names = set(re.findall(r"[A-Za-z_]\w*", expr)) - {"defined"}
    if not names or not names <= set(knobs):
        return None
    e = re.sub(r"defined\s*\(?\s*(\w+)\s*\)?", lambda m: "1" if m.group(1) in knobs else "0", expr)
    for k, v in knobs.items():
        e = re.sub(rf"\b{k}\b", str(v), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    e = re.sub(r"//.*", "", e)
    return bool(eval(e))


def process(lines, knobs):
    out = []
    # stack entries: (kind, keep_this_branch, taken_any, emit_directives)
    stack = []

    def active():
        return all(s[1] for s in stack)

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if active():
                out.append(ln)
            i += 1
            continue
        d, rest = m.group(1), m.group(2).strip()
        rest = re.sub(r"//.*", "", rest).strip()
        if d in ("ifndef", "ifdef", "if"):
            if d == "ifndef" and rest in knobs:
                # the default-value block: skip through its #endif
                j = i + 1
                depth = 1
                while depth:
                    t = lines[j].strip()
                    if re.match(r"#\s*if", t):
                        depth += 1
                    elif re.match(r"#\s*endif", t):
                        depth -= 1
                    j += 1
                i = j
                continue
            expr = rest if d == "if" else (f"defined({rest})" if d == "ifdef" else f"!defined({rest})")
            v = cond_value(expr, knobs)
            if v is None:
                stack.append(["keep", True, True, True])
                if active():
                    out.append(ln)
            else:
                stack.append(["eval", v, v, False])
        elif d == "elif":
            top = stack[-1]
            if top[0] == "keep":
                if all(x[1] for x in stack[:-1]):
                    out.append(ln)
            else:
                v = cond_value(rest, knobs)
                if v is None:
                    raise SystemExit(f"line {i + 1}: #elif on other macros after an evaluated #if")
                top[1] = (not top[2]) and v
                top[2] = top[2] or v
        elif d == "else":
            top = stack[-1]
            if top[0] == "keep":
                if all(x[1] for x in stack[:-1]):
                    out.append(ln)
            else:
                top[1] = not top[2]
                top[2] = True
        elif d == "endif":
            top = stack.pop()
            if top[0] == "keep" and active():
                out.append(ln)
        i += 1
    res = []
    for ln in out:  # uses in code (not in // comments) become the value
        code, sep, com = ln.partition("//")
        for k, v in knobs.items():
            code = re.sub(rf"\b{k}\b", str(v), code)
        res.append(code + sep + com)
    return "\n".join(res)


def main():
    path = sys.argv[1]
    knobs = {}
    for a in sys.argv[2:]:
        k, v = a.split("=")
        knobs[k] = int(v)
    lines = open(path).read().split("\n")
    open(path, "w").write(process(lines, knobs))


if __name__ == "__main__":
    main()
