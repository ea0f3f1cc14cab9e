#!/usr/bin/env python3
"""A small unifdef: resolve the preprocessor conditionals of the kernel
sources whose value is fixed by the given macro settings, in place.

  python scripts/unifdef.py -DRTW_BVH4=0 -DRTW_SORT_DPP=1 -URTW_FOO file...

A condition is resolved only when every identifier in it is one of the given
macros (or `defined(X)` of one); any other conditional line is kept as it
is, and so is its body (its nested conditionals are still resolved).  Used to
prune the A/B variants DESIGN.md records as measured and rejected: the
pruned build's device assembly is compared with the previous build's, so the
removal is checked to change no instruction.
"""
from __future__ import annotations

import re
import sys

TOKEN = re.compile(r"\s*(defined|\d+[uUlL]*|[A-Za-z_]\w*|&&|\|\||==|!=|<=|>=|[()!<>+\-*])")


class Unknown(Exception):
    pass


def evaluate(expr: str, known: dict[str, int | None]) -> int:
    """Value of a #if expression over `known` (None = undefined); raises
    Unknown when the expression names anything else."""
    expr = re.sub(r"//.*$", "", expr)
    expr = re.sub(r"/\*.*?\*/", "", expr).strip()
    toks, pos = [], 0
    while pos < len(expr):
        m = TOKEN.match(expr, pos)
        if not m:
            raise Unknown(expr)
        toks.append(m.group(1))
        pos = m.end()
    out = []
    i = 0
    while i < len(toks):
        t = toks[i]
        if t == "defined":
            if toks[i + 1] == "(":
                name, i = toks[i + 2], i + 4
            else:
                name, i = toks[i + 1], i + 2
            if name not in known:
                raise Unknown(name)
            out.append("1" if known[name] is not None else "0")
            continue
        if re.match(r"[A-Za-z_]", t):
            if t not in known or known[t] is None:
                raise Unknown(t)
            out.append(str(known[t]))
        elif t == "&&":
            out.append(" and ")
        elif t == "||":
            out.append(" or ")
        elif t == "!":
            out.append(" not ")
        else:
            out.append(re.sub(r"[uUlL]+$", "", t))
        i += 1
    return int(bool(eval("".join(out), {"__builtins__": {}})))


DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")


def process(lines: list[str], known) -> list[str]:
    """Resolved chains (every condition so far known) drop their directive
    lines and the bodies not taken; unresolved chains keep their lines, drop
    branches whose #elif is known false and turn a known-true #elif into the
    chain's #else."""
    out = []
    stack: list[dict] = []

    def parents_keep():
        return all(s["keep"] for s in stack[:-1])

    for line in lines:
        m = DIRECTIVE.match(line)
        # a directive continued over several lines stays as it is
        if not m or line.rstrip().endswith("\\"):
            if all(s["keep"] for s in stack):
                out.append(line)
            continue
        kind, rest = m.group(1), m.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            try:
                if kind == "if":
                    v = evaluate(rest, known)
                else:
                    name = rest.split()[0]
                    if name not in known:
                        raise Unknown(name)
                    v = int((known[name] is not None) == (kind == "ifdef"))
                stack.append({"resolved": True, "taken": bool(v), "keep": bool(v)})
            except Unknown:
                stack.append({"resolved": False, "keep": True, "rest_dead": False})
                if parents_keep():
                    out.append(line)
            continue
        top = stack[-1]
        if kind == "elif":
            if top["resolved"]:
                if top["taken"]:
                    top["keep"] = False
                    continue
                try:
                    v = evaluate(rest, known)
                    top["taken"] = top["keep"] = bool(v)
                except Unknown:
                    stack[-1] = {"resolved": False, "keep": True, "rest_dead": False}
                    if parents_keep():
                        out.append(re.sub(r"#(\s*)elif", r"#\1if", line, count=1))
                continue
            if top["rest_dead"]:
                top["keep"] = False
                continue
            try:
                v = evaluate(rest, known)
            except Unknown:
                top["keep"] = True
                if parents_keep():
                    out.append(line)
                continue
            if v:
                top["keep"] = True
                top["rest_dead"] = True
                if parents_keep():
                    out.append(line[: line.index("#")] + "#else\n")
            else:
                top["keep"] = False
            continue
        if kind == "else":
            if top["resolved"]:
                top["keep"] = not top["taken"]
                top["taken"] = True
                continue
            top["keep"] = not top["rest_dead"]
            if top["keep"] and parents_keep():
                out.append(line)
            continue
        # endif
        stack.pop()
        if not top["resolved"] and all(s["keep"] for s in stack):
            out.append(line)
    assert not stack, "unbalanced conditionals"
    return out


def main(argv):
    known: dict[str, int | None] = {}
    files = []
    for a in argv:
        if a.startswith("-D"):
            name, _, val = a[2:].partition("=")
            known[name] = int(val) if val else 1
        elif a.startswith("-U"):
            known[a[2:]] = None
        else:
            files.append(a)
    for f in files:
        with open(f) as fh:
            lines = fh.readlines()
        new = process(lines, known)
        if new != lines:
            with open(f, "w") as fh:
                fh.writelines(new)
            print(f"{f}: {len(lines)} -> {len(new)} lines")


if __name__ == "__main__":
    main(sys.argv[1:])
