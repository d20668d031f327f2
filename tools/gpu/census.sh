set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/block_timing.py > gpurun_out/block_timing.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_census.py > gpurun_out/gemm_census.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_kernels.py --only dw > gpurun_out/kb_dw.log 2>&1
echo rc=$?
