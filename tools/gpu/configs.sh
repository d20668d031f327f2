#!/bin/bash
# The other BASELINE configurations on the current build: long history (T=15, b64) and 456x456 (T=6, b128, bf16).
source "$(dirname "$0")/step.sh"
TAIL=1 run_step cfg_t15 400 python -u bench.py --seq_len 15 --batch_per_gpu 64 --steps 10 --warmup 3
TAIL=1 run_step cfg_456 400 python -u bench.py --height 456 --width 456 --steps 10 --warmup 3
