#!/bin/bash
# Kernel traces of the eager bench step for the previous build (build/base) and the current one, same box.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
rm -rf gpurun_out/trA gpurun_out/trB
RT1_HIP_SO=build/base/$SO TAIL=1 run_step trA 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trA -o run \
    -- python3 bench.py --steps 6 --warmup 2 --graph off --no_check
TAIL=1 run_step trB 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trB -o run \
    -- python3 bench.py --steps 6 --warmup 2 --graph off --no_check
