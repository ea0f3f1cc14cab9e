"""Per-kernel register / scratch / occupancy table from a hipcc
-Rpass-analysis=kernel-resource-usage log.

  hipcc ... --offload-device-only -Rpass-analysis=kernel-resource-usage 2> ru.txt
  python scripts/resource_usage.py ru.txt [name-substring]
"""
import re
import subprocess
import sys

rows, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?): (\S+) \[-Rpass", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, n in zip(rows, names):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if flt not in n:
        continue
    print(f"{n:44s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} SGPR {r.get('TotalSGPRs', '?'):>4} "
          f"Vspill {r.get('VGPRs Spill', '?'):>4} Sspill {r.get('SGPRs Spill', '?'):>4} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} occ {r.get('Occupancy [waves/SIMD]', '?'):>2} "
          f"LDS {r.get('LDS Size [bytes/block]', '?')}")
