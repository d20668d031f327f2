#!/bin/bash
# se_rowmat forward tile threshold: in-tree (32-frame tiles from 200 workgroups) vs fwd300 (from 300) vs HEAD build.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step se_ab5_fwd300 300 python -u tools/bench_se.py --ab build/fwd300/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step se_ab5_head 300 python -u tools/bench_se.py --ab build/head2/_rt1_hip.cpython-310-x86_64-linux-gnu.so
