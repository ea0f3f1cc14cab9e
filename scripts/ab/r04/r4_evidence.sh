#!/bin/bash
# round-4 final evidence in one call: part 1 (GPU suite, rocprof, fp64 PMC records), the records copied
# under profiles/pmc/ so the bench lines carry them, then part 2 (fp32 records, bench / config / fp32 /
# full-size lines)
set -e
tag=$1
bash scripts/r4_evidence_a.sh $tag
cp gpurun_out/pmc/*_$tag.json profiles/pmc/
bash scripts/r4_evidence_b.sh $tag
