#!/bin/bash
# se_rowmat variants vs the in-tree build (16-frame tiles below 512 workgroups, V prefetched): 32-frame tiles from 256
# workgroups up (rm256), always 32-frame tiles (rmft32), no V prefetch (rmnopf).
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
for v in rm256 rmft32 rmnopf rm256; do
  run_step se_ab_$v 300 python -u tools/bench_se.py --ab build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so
done
