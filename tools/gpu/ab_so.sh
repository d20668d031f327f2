#!/bin/bash
# Same-box A/B of two builds of the extension: bench.py with the default in-tree .so vs RT1_HIP_SO=$BASE_SO, alternated.
#   BASE_SO=build/base/_rt1_hip.cpython-310-x86_64-linux-gnu.so TAG=x bash tools/gpu/ab_so.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-abso}
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/abso_${TAG}_base_$rep.log 2>&1 || { echo "base failed"; tail -5 gpurun_out/abso_${TAG}_base_$rep.log; exit 1; }
  echo "base rep$rep: $(tail -1 gpurun_out/abso_${TAG}_base_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/abso_${TAG}_new_$rep.log 2>&1 || { echo "new failed"; tail -5 gpurun_out/abso_${TAG}_new_$rep.log; exit 1; }
  echo "new  rep$rep: $(tail -1 gpurun_out/abso_${TAG}_new_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
