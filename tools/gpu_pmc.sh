#!/bin/bash
# kernel tests + per-layer microbench + SQ counters for two representative depthwise layers
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_backbone_gpu.py -q -s > gpurun_out/pytest_enc.log 2>&1; rc=$?
grep -E "passed|failed|encoder fwd|grad err" gpurun_out/pytest_enc.log | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed $rc"; exit 1; fi
timeout -k 10 600 python tools/bench_kernels.py --frames 768 --res 300 > gpurun_out/kbench.log 2>&1 || { echo "kbench failed $?"; tail -5 gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
B=${PMC_BLOCKS:-2,14}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d gpurun_out/pmc1 -o pmc -- python3 tools/bench_kernels.py --blocks $B --iters 2 > gpurun_out/pmc1.log 2>&1 || { echo "pmc1 failed $?"; tail -5 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU \
  --output-format csv -d gpurun_out/pmc2 -o pmc -- python3 tools/bench_kernels.py --blocks $B --iters 2 > gpurun_out/pmc2.log 2>&1 || { echo "pmc2 failed $?"; tail -5 gpurun_out/pmc2.log; exit 1; }
find gpurun_out/pmc1 gpurun_out/pmc2 -name "*.csv" | head
