#!/bin/bash
# end-of-session checkpoint: GPU suite + smoke + bench, then the cumulative same-box A/B vs the session start commit
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAIL=3 run_step final_suite 900 env TAG=r6s3c PROF=0 bash tools/gpu/suite.sh
REPS="1 2 3" BASE_TREE=build/base_tree TAG=sessf STEPS=30 TAIL=8 run_step sessf_ab 700 bash tools/gpu/ab_tree.sh
