#!/bin/bash
# driver hooks (build import + smoke), LAVA BC training on the GPU, GPU suite, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed $?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python train_lava.py --collect 24 --steps 150 --batch_size 64 --log_every 50 --ckpt gpurun_out/lava/last.pt --eval_episodes 4 > gpurun_out/lava.log 2>&1 || { echo "lava failed $?"; tail -20 gpurun_out/lava.log; exit 1; }
tail -4 gpurun_out/lava.log
rm -rf gpurun_out/lava
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed $?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
