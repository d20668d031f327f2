#!/bin/bash
# Re-tune the library GEMMs of the current step (PyTorch TunableOp) into gpurun_out/tunableop_results<dev>.csv, then
# A/B bench.py on the in-tree recorded solutions (tuning/) vs the fresh ones, alternated on the same box.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 900 python -u bench.py --steps 2 --warmup 2 --no_check > gpurun_out/tunable_retune.log 2>&1 || { echo "tune failed $?"; tail -20 gpurun_out/tunable_retune.log; exit 1; }
wc -l gpurun_out/tunableop_results*.csv
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tunable_old_$rep.log 2>&1 || exit 1
  echo "old rep$rep: $(tail -1 gpurun_out/tunable_old_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tunable_new_$rep.log 2>&1 || { echo "new failed"; tail -20 gpurun_out/tunable_new_$rep.log; exit 1; }
  echo "new rep$rep: $(tail -1 gpurun_out/tunable_new_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
