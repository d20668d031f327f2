#!/bin/bash
# SQ counters of every kernel of ONE eager bench step (300x300, b128): instruction mix, wait fractions, LDS bank
# conflicts, occupancy.  One counter group per rocprofv3 --pmc pass (<= 8 SQ, <= 2 GRBM per pass), each under its own
# hard limit; tools/pmc_step_sq.py aggregates the last step per kernel.
#   TAG=sq1 bash tools/gpu/pmc_sq_step.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sq}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
run() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o pmc -- python3 bench.py --steps 2 --warmup 1 --graph off --no_check ${BENCH_ARGS} \
    > gpurun_out/${TAG}_$name.log 2>&1 || { echo "pmc $name failed $?"; tail -5 gpurun_out/${TAG}_$name.log; return 1; }
  echo "pass $name done"
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run b SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 1
find gpurun_out -path "gpurun_out/${TAG}_*" -name "*.db" -delete
python3 tools/pmc_step_sq.py gpurun_out/${TAG}_a gpurun_out/${TAG}_b > gpurun_out/${TAG}_summary.txt 2>&1
head -40 gpurun_out/${TAG}_summary.txt
