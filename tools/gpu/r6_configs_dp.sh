#!/bin/bash
# other BASELINE configurations + the segmented graph-DP step on a world-1 RCCL communicator (the N > 1 path)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAIL=1 run_step r6s3_cfg_t15 400 python -u bench.py --seq_len 15 --batch_per_gpu 64 --steps 10 --warmup 3
TAIL=1 run_step r6s3_cfg_456 400 python -u bench.py --height 456 --width 456 --steps 10 --warmup 3
TAIL=1 run_step r6s3_native1 400 python -u bench.py --steps 20 --warmup 5 --comm native
TAIL=1 run_step r6s3_graph1 400 python -u bench.py --steps 20 --warmup 5
run_step r6s3_film_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_film_gpu.py
run_step r6s3_film_bench 300 python -u tools/bench_film.py
