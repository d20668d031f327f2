#!/bin/bash
# LDS-tiled pw_z_finish + se_rowmat (16-frame tiles, V prefetched under the partial sums): numerics tests, isolated
# A/Bs against the committed HEAD build, bench A/B; then the idle-communicator stream-priority check.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/head2/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step zf_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pwgemm_gpu.py \
    tests/test_backbone_gpu.py -k "pw_z or se_fused or pwgemm or pw_"
run_step zf_ab 300 python -u tools/bench_zprep.py --ab $BASE_SO
run_step se_ab 300 python -u tools/bench_se.py --ab $BASE_SO
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step zf_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step zf_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
for rep in 1 2; do
  RT1_DP_DIAG=comminit TAIL=1 run_step dl_comminit_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=comminit RT1_COMM_STREAM=normal TAIL=1 run_step dl_comminit_normal_$rep 300 python -u bench.py --steps 20 --warmup 5
done
