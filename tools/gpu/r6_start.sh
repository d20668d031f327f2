#!/bin/bash
# Round-6 opening measurements: the one-graph bench, the segmented graph-DP step on a world-1 RCCL communicator
# (--comm native: the same path the N>1 runs take), then SQ counters of every kernel of one eager step.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step r6_bench_graph 300 python -u bench.py --steps 20 --warmup 5
run_step r6_bench_native1 300 python -u bench.py --steps 20 --warmup 5 --comm native
TAG=r6sq run_step r6_pmc_sq 700 bash tools/gpu/pmc_sq_step.sh
