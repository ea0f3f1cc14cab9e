#!/bin/bash
# Scratch spills of one kernel in an ISA file (hipcc -S): each spill store /
# reload with the instructions that define the spilled register just before.
#   scripts/spills.sh KS.s KERNEL-SUBSTRING
f=$1; k=$2
start=$(grep -n "^_Z.*$k.*:" "$f" | head -1 | cut -d: -f1)
awk -v s="$start" 'NR>=s' "$f" | awk '/s_endpgm/{print; exit} {print}' > /tmp/spill_fn.s
echo "function lines: $(wc -l < /tmp/spill_fn.s); loop header: $(grep -n 'Loop Header' /tmp/spill_fn.s | head -1)"
grep -nE "scratch_(store|load)" /tmp/spill_fn.s || echo "no scratch spills"
