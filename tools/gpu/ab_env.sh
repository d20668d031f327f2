#!/bin/bash
# Same-box A/B of a switch: optional targeted GPU tests, then bench.py with the switch at each of $AB_VALUES (default
# "0 1") alternated.  AB_ENV is an ops/switches.py name (run as RT1_AB=<name>=<value>) or a whole RT1_* / HIP_* /
# DEBUG_CLR_* runtime variable.
#   TESTS="tests/test_pwgemm_gpu.py" K="pw_bwd_z" AB_ENV=pw_bwd_z TAG=x bash tools/gpu/ab_env.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS ${K:+-k "$K"} \
    > gpurun_out/ab_tests_$TAG.log 2>&1 || { echo "tests failed $?"; grep -E "FAILED|Error|assert" gpurun_out/ab_tests_$TAG.log | head -30; tail -30 gpurun_out/ab_tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/ab_tests_$TAG.log
fi
for rep in 1 2; do
  for v in ${AB_VALUES:-0 1}; do
    case "$AB_ENV" in RT1_*|HIP_*|DEBUG_CLR_*) setting="$AB_ENV=$v" ;; *) setting="RT1_AB=$AB_ENV=$v" ;; esac
    env "$setting" timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/ab_${TAG}_${v}_$rep.log 2>&1 || { echo "bench $v failed $?"; tail -20 gpurun_out/ab_${TAG}_${v}_$rep.log; exit 1; }
    echo "$AB_ENV=$v rep$rep: $(tail -1 gpurun_out/ab_${TAG}_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
