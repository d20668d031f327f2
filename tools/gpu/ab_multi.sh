#!/bin/bash
# Same-box A/B of several environment settings on bench.py, alternated over 2 reps:
#   VARIANTS="base:RT1_X=0 new:RT1_X=1" TAG=x bash tools/gpu/ab_multi.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
TAG=${TAG:-abm}
for rep in 1 2; do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/abm_${TAG}_${name}_$rep.log 2>&1 || { echo "bench $name failed $?"; tail -20 gpurun_out/abm_${TAG}_${name}_$rep.log; exit 1; }
    echo "$name ($envs) rep$rep: $(tail -1 gpurun_out/abm_${TAG}_${name}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
