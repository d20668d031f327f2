#!/bin/bash
# Fused-SE data-parallel discrepancy probes (2 gloo ranks on one GPU, tools/dp_gpu_check.py): eager-vs-eager and
# graph-vs-eager with the SE debug flags (pool / h / gate changed since the forward, se_bwd re-run mismatch), the
# local (pre-all-reduce) gradient comparison, and one run with the caching allocator off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/sedbg
export PYTHONPATH=$PWD
port=29561
run() {
    local name=$1 mode=$2; shift 2
    port=$((port + 1))
    timeout -k 10 200 env "$@" python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/dp_gpu_check.py $mode > gpurun_out/sedbg/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    grep -E "^step|mismatch|local grad|grad bucket" gpurun_out/sedbg/$name.log | head -40
    # 0 = equal, 1 = torchrun reports a rank's non-zero exit (2 = mismatch); anything else: stop here
    if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
    if grep -qE "Segmentation|core dumped|HSA_STATUS|hipError|Memory access fault" gpurun_out/sedbg/$name.log; then
        echo "fault in $name"; exit 3
    fi
    return 0
}
run e2a --eager2 RT1_SE_FUSED=force RT1_SE_DEBUG=1
run ga --graph RT1_SE_FUSED=force RT1_SE_DEBUG=1
run e2b --eager2 RT1_SE_FUSED=force RT1_SE_DEBUG=1
run nocache --eager2 RT1_SE_FUSED=force RT1_SE_DEBUG=1 PYTORCH_NO_HIP_MEMORY_CACHING=1
run gb --graph RT1_SE_FUSED=force
