#!/bin/bash
# SQ counters of the depthwise kernels on representative layers (block 3: k3 75x75x192, block 14: k5 19x19x816).
# PMC_TOOL=tools/bench_dw_fused.py profiles the fused backward instead.
# One counter group per rocprofv3 run (each within the per-block limits), each under its own hard time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcdw}
B=${PMC_BLOCKS:-3,14}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o pmc -- python3 ${PMC_TOOL:-tools/bench_kernels.py} --blocks $B --iters 2 \
    > gpurun_out/${TAG}_$name.log 2>&1 || { echo "pmc $name failed $?"; tail -5 gpurun_out/${TAG}_$name.log; return 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU || exit 1
if grep -q "SQ_ACTIVE_INST_VALU" gpurun_out/${TAG}_counters.txt && grep -q "SQ_INSTS_VMEM_RD" gpurun_out/${TAG}_counters.txt; then
  run c SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 1
fi
find gpurun_out -path "gpurun_out/${TAG}_*" -name "*.db" -delete
python3 tools/pmc_summary.py gpurun_out/${TAG}_a gpurun_out/${TAG}_b $( [ -d gpurun_out/${TAG}_c ] && echo gpurun_out/${TAG}_c ) > gpurun_out/${TAG}_summary.txt 2>&1
grep -E "dw_" gpurun_out/${TAG}_summary.txt | head -40
