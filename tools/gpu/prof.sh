#!/bin/bash
# rocprofv3 kernel trace + stats of the 1-GPU bench (eager step, so each kernel is a dispatch) -> markdown summary
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${PROF_TAG:-prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --steps ${PROF_STEPS:-3} --warmup 2 --graph off ${BENCH_ARGS} > gpurun_out/$TAG.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/$TAG.log; exit 1; }
tail -1 gpurun_out/$TAG.log
find gpurun_out/$TAG -name "*.db" -delete; find gpurun_out/$TAG -name "*kernel_trace.csv" -delete -o -name "*agent_info*" -delete; python3 tools/rocprof_summary.py gpurun_out/$TAG --top ${PROF_TOP:-60} --out gpurun_out/$TAG.md --title "${PROF_TITLE:-rocprofv3 kernel summary}" && head -70 gpurun_out/$TAG.md
