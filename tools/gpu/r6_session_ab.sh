#!/bin/bash
# cumulative same-box A/B: the session-3 start commit (build/base_tree) vs this tree, 4 interleaved pairs
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_TREE=build/base_tree TAG=sess STEPS=30 TAIL=10 run_step sess_ab 1000 bash tools/gpu/ab_tree.sh
