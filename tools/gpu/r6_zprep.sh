#!/bin/bash
# pw_z_prep with LDS-staged We chunks: numerics tests, isolated A/B vs the HEAD build, bench A/B.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/head/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step zp_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pwgemm_gpu.py
run_step zp_ab 300 python -u tools/bench_zprep.py --ab $BASE_SO
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step zp_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step zp_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
RT1_DP_DIAG=comminit TAIL=1 run_step dj_comminit 300 python -u bench.py --steps 20 --warmup 5
TAIL=1 run_step dj_graph 300 python -u bench.py --steps 20 --warmup 5
for rep in 1 2; do
  TAIL=1 run_step dk_native_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  RT1_DP_DIAG=keepcache TAIL=1 run_step dk_keepcache_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
done
