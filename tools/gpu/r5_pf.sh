#!/bin/bash
# dw forward with the next tile's loads in flight (RT1_DW_FWD_PF): numerics on the default build, then per-layer
# forward times for PF = 0 / 2 / 4 / 6 builds, alternated twice
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step pf_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backbone_gpu.py -k "dwconv_fwd_bwd"
for rep in 1 2; do
  for v in pf0 pf2 pf4 pf6; do
    so=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so
    [ "$v" = pf4 ] && so=pytorch_rt1_for_distributed_training_amd/_rt1_hip.cpython-310-x86_64-linux-gnu.so
    RT1_HIP_SO=$so run_step pf_${v}_$rep 200 python -u tools/bench_dw_phases.py --fwd_only --tag $v
  done
done
