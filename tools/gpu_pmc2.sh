#!/bin/bash
# SQ counters for the depthwise kernels of one block (KB_BLOCKS), 2 passes, summarised per kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${KB_BLOCKS:-14}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --output-format csv -d gpurun_out/pmcA -o pmc -- python3 tools/bench_kernels.py --blocks $B --iters 2 > gpurun_out/pmcA.log 2>&1 || { echo "pmcA failed $?"; tail -5 gpurun_out/pmcA.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM \
  --output-format csv -d gpurun_out/pmcB -o pmc -- python3 tools/bench_kernels.py --blocks $B --iters 2 > gpurun_out/pmcB.log 2>&1 || { echo "pmcB failed $?"; tail -5 gpurun_out/pmcB.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_summary.txt && cat gpurun_out/pmc_summary.txt
