#!/bin/bash
# rocprofv3 memory-copy + kernel trace of the eager 1-GPU bench step: where do the per-step __amd_rocclr_copyBuffer
# dispatches come from (direction / size of every hipMemcpy*)?  -> gpurun_out/memcpy_trace.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/mct -o run -- python3 bench.py --steps 3 --warmup 2 --graph off > gpurun_out/mct.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/mct.log; exit 1; }
tail -1 gpurun_out/mct.log
python3 tools/memcpy_report.py gpurun_out/mct > gpurun_out/memcpy_trace.txt && cat gpurun_out/memcpy_trace.txt
find gpurun_out/mct -name "*.db" -delete; gzip -f gpurun_out/mct/*kernel_trace.csv
