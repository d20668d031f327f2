#!/bin/bash
# depthwise forward sweep on the high-resolution layers: grid caps x staging-load variants (tools/bench_kernels.py)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in default su8 su2; do
  for fb in 1024 2048 4096 8192; do
    if [ $so = default ]; then unset RT1_HIP_SO; else export RT1_HIP_SO=build/$so/_rt1_hip.cpython-310-x86_64-linux-gnu.so; fi
    timeout -k 10 200 python tools/bench_kernels.py --frames 768 --res 300 --blocks 0,1,2,3,5,8 --fwd_blocks $fb --iters 5 > gpurun_out/dwf_${so}_$fb.log 2>&1 || { echo "fail $so $fb"; tail -5 gpurun_out/dwf_${so}_$fb.log; exit 1; }
    echo "== $so fwd_blocks=$fb"; grep -E "^ +[0-9]+ " gpurun_out/dwf_${so}_$fb.log | awk '{print $1, $6, $8, $9, $11}'
  done
done
