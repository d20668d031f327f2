#!/bin/bash
# Kernel trace of the 1-GPU hipGraph bench step: span vs kernel-busy union per replayed step (launch / dependency
# bubbles inside the graph), small-kernel census.  -> gpurun_out/r6_gaps.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/gaps.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/gaps.log; exit 1; }
tail -1 gpurun_out/gaps.log
f=$(find gpurun_out/gaps -name "*kernel_trace.csv" | head -1)
python3 tools/graph_gaps.py "$f" --steps 4 > gpurun_out/r6_gaps.txt && cat gpurun_out/r6_gaps.txt
find gpurun_out/gaps -name "*.db" -delete; gzip -f gpurun_out/gaps/*/*kernel_trace.csv gpurun_out/gaps/*kernel_trace.csv 2>/dev/null; true
