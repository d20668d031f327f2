#!/bin/bash
# pw_tall project GEMMs (blocks 8-17) on the HEAD build (build/base) and the working tree
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
RT1_HIP_SO=build/base/$SO TAIL=12 run_step tallk_base 300 python -u tools/bench_proj_prologue.py --blocks 8,9,13,14
TAIL=12 run_step tallk_new 300 python -u tools/bench_proj_prologue.py --blocks 8,9,13,14
