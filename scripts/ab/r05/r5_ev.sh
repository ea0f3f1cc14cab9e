#!/bin/bash
# round 5 evidence in ONE call (tag $1): GPU suite, rocprof of the default
# bench command, PMC records of T, C2, C3, C5 and the fp32 T, C2, C3, C5 (in
# profiles/pmc/ on the box before the lines run), the default T line, config
# lines, fp32 lines, full-size C4 / C5 lines
set -e
tag=$1
bash scripts/ab/r05/r5_ev1.sh $tag
cp gpurun_out/pmc/*_$tag.json profiles/pmc/
bash scripts/ab/r05/r5_ev2.sh $tag
# where the lane time goes (the -DRTW_PROF build of the same sources)
bash scripts/prof_sections.sh
