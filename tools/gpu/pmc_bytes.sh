#!/bin/bash
# HBM bytes per kernel of the eager bench step: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (TCC
# counter limit), each under its own hard time limit; tools/pmc_summary.py averages per kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcb}
run() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o pmc -- python3 bench.py --steps 2 --warmup 1 --graph off --no_check \
    > gpurun_out/${TAG}_$name.log 2>&1 || { echo "pmc $name failed $?"; tail -5 gpurun_out/${TAG}_$name.log; return 1; }
  echo "pass $name done"
}
run f FETCH_SIZE || exit 1
run w WRITE_SIZE || exit 1
find gpurun_out -path "gpurun_out/${TAG}_*" -name "*.db" -delete
python3 tools/pmc_summary.py gpurun_out/${TAG}_f gpurun_out/${TAG}_w > gpurun_out/${TAG}_summary.txt 2>&1
head -5 gpurun_out/${TAG}_summary.txt
