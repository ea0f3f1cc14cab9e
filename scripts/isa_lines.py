"""Static VALU cost of one kernel by source line (hipcc -S -g1 ISA).

  python scripts/isa_lines.py KS.s FUNCTION-SUBSTRING [TOP] [--outer FILE]

--outer FILE charges each instruction to the OUTERMOST line of FILE in its
inline chain (e.g. --outer rtw_kernels.hip: which call site of the kernel
body the instruction belongs to -- camera sample, world walk, sort prefix,
shading) instead of the innermost line.  That view found the counting
sort's block prefix (~67 VALU per wave-iteration, EXPERIMENTS.md).

Each v_* instruction is weighted by its measured issue cost on gfx950
(scripts/valu_rates.hip, profiles/r01/valu_rates.log: fp64 ~4.7 cycles per wave
instruction, fp32 / integer ~2.6, fp64 rcp / rsq / sqrt ~17) and charged to the
innermost source line its .loc names.  A static map -- it says where the
kernel's instructions are, not how often each runs.
"""
import re
import sys
from collections import defaultdict

args = sys.argv[1:]
outer = None
if "--outer" in args:
    k = args.index("--outer")
    outer = args[k + 1]
    del args[k:k + 2]
path, fname = args[0], args[1]
top = int(args[2]) if len(args) > 2 else 40
lines = open(path).read().splitlines()
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(fname) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))

TRANS64 = ("v_rcp_f64", "v_rsq_f64", "v_sqrt_f64")


def cost(op):
    if op.startswith(TRANS64):
        return 17.0
    if "_f64" in op or op.startswith(("v_div_fmas_f64", "v_div_scale_f64", "v_trig_preop", "v_ldexp_f64")):
        return 4.7
    return 2.6


cur = "?"
by_line = defaultdict(lambda: [0, 0.0, 0])
tot = [0, 0.0]
for l in lines[start:end]:
    s = l.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        if outer:  # the outermost frame of `outer` in the comment's inline chain
            frames = re.findall(re.escape(outer) + r":(\d+)", l)
            cur = f"{outer}:{frames[-1]}" if frames else "(other)"
        continue
    m = re.match(r"(v_\w+)", s)
    if m:
        c = cost(m.group(1))
        b = by_line[cur]
        b[0] += 1
        b[1] += c
        if "_f64" in m.group(1):
            b[2] += 1
        tot[0] += 1
        tot[1] += c
print(f"{fname}: {tot[0]} VALU instructions, {tot[1]:.0f} weighted cycles")
for k, (n, c, f) in sorted(by_line.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{c:8.0f} {n:5d} f64 {f:4d}  {k}")
