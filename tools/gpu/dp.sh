#!/bin/bash
# Data-parallel rehearsals on ONE MI355X (2 ranks share cuda:0, collectives over gloo: RCCL refuses two ranks on
# one device): graph-DP vs eager-DP bitwise check, cross-rank parameter equality, and bench.py --gpus 2 spawning
# its own ranks.  Optional (DP_PROF=1): a kernel + memory-copy trace of each rank of the 2-rank bench rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dp}
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  tools/dp_gpu_check.py --graph > gpurun_out/${TAG}_graph_check.log 2>&1 || { echo "graph-DP check failed $?"; tail -40 gpurun_out/${TAG}_graph_check.log; exit 1; }
grep -E "^step|grad bucket" gpurun_out/${TAG}_graph_check.log
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  tools/dp_gpu_check.py > gpurun_out/${TAG}_rank_check.log 2>&1 || { echo "cross-rank check failed $?"; tail -30 gpurun_out/${TAG}_rank_check.log; exit 1; }
grep -E "^losses" gpurun_out/${TAG}_rank_check.log
RT1_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --batch_per_gpu 32 --steps 5 --warmup 3 \
  > gpurun_out/${TAG}_bench2.log 2>&1 || { echo "bench --gpus 2 failed $?"; tail -30 gpurun_out/${TAG}_bench2.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench2.log
if [ "${DP_PROF:-0}" = "1" ]; then
  P=$((29600 + RANDOM % 200))
  for r in 0 1; do
    RT1_DIST_BACKEND=gloo RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$P \
      timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_trace_r$r -o run \
      -- python3 bench.py --gpus 2 --batch_per_gpu 32 --steps 3 --warmup 3 > gpurun_out/${TAG}_trace_r$r.log 2>&1 &
  done
  wait -n || { echo "traced rank failed"; exit 1; }
  wait -n || { echo "traced rank failed"; exit 1; }
  tail -1 gpurun_out/${TAG}_trace_r0.log
  find gpurun_out/${TAG}_trace_r0 gpurun_out/${TAG}_trace_r1 -name "*.db" -delete
fi
exit 0
