#!/bin/bash
# Shared helper for multi-step GPU sessions: run_step NAME SECONDS CMD... runs one step under its own time limit with
# its output in gpurun_out/NAME.log, prints its tail, and ends the whole session (exit code of the step) after a
# crash, an abort or a time limit -- nothing more runs on the GPU after those.  Plain failures (a test that fails,
# a mismatch exit code) let the session continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
run_step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    tail -n "${TAIL:-15}" "gpurun_out/$name.log"
    echo "=== $name rc=$rc"
    case $rc in
        124|134|137|139) echo "stopping the session after $name (rc=$rc)"; exit $rc ;;
    esac
    if grep -qE "Memory access fault|HSA_STATUS_ERROR|core dumped" "gpurun_out/$name.log"; then
        echo "GPU fault in $name: stopping"; exit 3
    fi
    return 0
}
