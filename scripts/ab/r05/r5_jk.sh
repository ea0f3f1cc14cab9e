#!/bin/bash
# round 5, calls j + k in one box: the shared-GPU rehearsal, then the overlap A/B
set -e
bash scripts/ab/r05/r5_j.sh
bash scripts/ab/r05/r5_k.sh
