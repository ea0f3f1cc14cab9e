"""Where a kernel's VGPR pressure peaks: backward liveness over the ISA of one
function (hipcc -S -g1, so .loc lines map instructions to source lines).

  python scripts/vgpr_live.py KS.s FUNCTION-SUBSTRING [TOP [INSTRUCTION#]]

Prints the instructions with the most live VGPRs, the source line each sits
on, and for the hottest one the live registers with the source line of their
reaching definition.  Approximate: a write is taken as a full definition
(exec-masked partial writes are not modelled) -- a map of where pressure
comes from, not the allocator's exact count.
"""
import re
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if a != "--sgpr"]
SGPR = "--sgpr" in sys.argv  # analyse SGPRs instead (s_* defs, v_cmp/readlane/carry-out defs)
sys.argv = [sys.argv[0]] + args
path, fname = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
lines = open(path).read().splitlines()

files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]

# the function body
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(fname) + r"\S*:", l) or
             (fname in l and l.rstrip().endswith(":") and not l.startswith("\t")))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))

REG = re.compile(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]") if SGPR else re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
NODEF = ("_store", "ds_write", "s_", "v_cmp_", "v_cmpx_", "v_readlane", "v_readfirstlane", "buffer_atomic",
         "global_atomic", "flat_atomic", "ds_add", "ds_max", "ds_min")


def regs(text):
    out = []
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


insts = []  # (op, defs, uses, srcline, text)
labels = {}
cur_loc = "?"
for i in range(start + 1, end):
    l = lines[i].split(";")[0].strip()
    if not l:
        continue
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur_loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    if l.endswith(":"):
        labels[l[:-1]] = len(insts)
        continue
    if l.startswith("."):
        continue
    parts = l.split(None, 1)
    op = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    operands = [o.strip() for o in re.split(r",(?![^\[]*\])", ops)] if ops else []
    defs, uses = [], []
    glc_ret = op.endswith("_rtn") or " glc" in ops or "sc0" in ops
    if SGPR:
        if op.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop",
                          "s_endpgm", "s_setprio", "s_sleep", "s_store", "s_atomic", "s_dcache", "s_sendmsg")) or \
                op.startswith(("v_", "ds_", "global_", "buffer_", "flat_", "scratch_")) and not (
                op.startswith(("v_cmp_", "v_cmpx_", "v_readlane", "v_readfirstlane")) and "_e64" in op or
                op.startswith(("v_readlane", "v_readfirstlane"))):
            # no SGPR def in the first operand; carry-out / scale defs in the second
            if op.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_div_scale", "v_mad_u64", "v_mad_i64",
                              "v_addc_co", "v_subb_co")) and len(operands) > 1:
                defs += regs(operands[1])
                for o in operands[:1] + operands[2:]:
                    uses += regs(o)
            else:
                for o in operands:
                    uses += regs(o)
        elif operands:
            defs += regs(operands[0])
            for o in operands[1:]:
                uses += regs(o)
        insts.append((op, set(defs), set(uses), cur_loc, l))
        continue
    if op.startswith(NODEF) and not (("atomic" in op) and glc_ret):
        for o in operands:
            uses += regs(o)
    elif op.startswith("v_writelane"):
        defs += regs(operands[0])
        uses += regs(operands[0])
    else:
        if operands:
            defs += regs(operands[0])
            for o in operands[1:]:
                uses += regs(o)
    insts.append((op, set(defs), set(uses), cur_loc, l))

n = len(insts)
succ = [[] for _ in range(n)]
for k, (op, d, u, loc, text) in enumerate(insts):
    tgt = text.split()[-1] if op.startswith(("s_branch", "s_cbranch")) else None
    if op == "s_endpgm":
        continue
    if op == "s_branch":
        succ[k].append(labels[tgt])
        continue
    if op.startswith("s_cbranch"):
        succ[k].append(labels[tgt])
    if k + 1 < n:
        succ[k].append(k + 1)

live_in = [set() for _ in range(n)]
changed = True
while changed:
    changed = False
    for k in range(n - 1, -1, -1):
        out = set()
        for s in succ[k]:
            out |= live_in[s]
        op, d, u, loc, text = insts[k]
        li = (out - d) | u
        if li != live_in[k]:
            live_in[k] = li
            changed = True

# reaching def's source line, per register, per instruction (forward, last def on any path)
rdef = [dict() for _ in range(n)]
pred = defaultdict(list)
for k in range(n):
    for s in succ[k]:
        pred[s].append(k)
changed = True
while changed:
    changed = False
    for k in range(n):
        inn = {}
        for p in pred[k]:
            for r, locs in rdef[p].items():
                inn.setdefault(r, set()).update(locs)
        op, d, u, loc, text = insts[k]
        for r in d:
            inn[r] = {loc}
        if inn != rdef[k]:
            rdef[k] = inn
            changed = True

order = sorted(range(n), key=lambda k: -len(live_in[k]))
print(f"{n} instructions; max live {'SGPRs' if SGPR else 'VGPRs'} {len(live_in[order[0]])}")
seen_loc = set()
shown = 0
for k in order:
    loc = insts[k][3]
    if loc in seen_loc:
        continue
    seen_loc.add(loc)
    print(f"  {len(live_in[k]):4d} live at #{k} {loc:24s} {insts[k][4][:70]}")
    shown += 1
    if shown >= top:
        break
k = int(sys.argv[4]) if len(sys.argv) > 4 else order[0]  # optional: instruction index to dump
by_loc = defaultdict(list)
for r in sorted(live_in[k]):
    locs = rdef[k - 1].get(r, {"(entry)"}) if k else {"(entry)"}
    by_loc[", ".join(sorted(locs))].append(r)
print(f"\nlive at #{k} ({insts[k][3]}), by defining source line:")
for loc, rs in sorted(by_loc.items(), key=lambda x: -len(x[1])):
    print(f"  {len(rs):3d}  {loc}   v{rs}")

# spill stores: which value (its defining source line) goes to which slot
spills = [k for k in range(n) if insts[k][0].startswith("scratch_store")]
if spills:
    print("\nspill stores (slot <- register defined at):")
    for k in spills:
        op, d, u, loc, text = insts[k]
        slot = re.search(r"offset:(\d+)", text)
        src = sorted(u)
        defs = set()
        for r in src:
            defs |= rdef[k - 1].get(r, {"(entry)"}) if k else {"(entry)"}
        print(f"  #{k:5d} {loc:24s} slot {slot.group(1) if slot else 0:>4}  v{src}  def at {', '.join(sorted(defs))}")
    reloads = defaultdict(list)
    for k in range(n):
        if insts[k][0].startswith("scratch_load"):
            slot = re.search(r"offset:(\d+)", insts[k][4])
            reloads[slot.group(1) if slot else "0"].append(insts[k][3])
    print("reloads per slot (source lines):")
    for sl, locs in sorted(reloads.items(), key=lambda x: int(x[0])):
        print(f"  slot {sl:>4}: {len(locs)} x  {', '.join(sorted(set(locs)))}")
