#!/bin/bash
# hipBLASLt solution tuning for the library GEMMs the step still issues (PyTorch TunableOp): one tuning run writes
# gpurun_out/tunableop_results.csv, then bench.py runs with tuning off reading that file vs without TunableOp.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 900 python -u bench.py --steps 2 --warmup 2 > gpurun_out/tunable_tune.log 2>&1 || { echo "tune failed $?"; tail -20 gpurun_out/tunable_tune.log; exit 1; }
ls -la gpurun_out/tunableop_results*.csv; wc -l gpurun_out/tunableop_results*.csv
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tunable_off_$rep.log 2>&1 || exit 1
  echo "off rep$rep: $(tail -1 gpurun_out/tunable_off_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tunable_on_$rep.log 2>&1 || { echo "on failed"; tail -20 gpurun_out/tunable_on_$rep.log; exit 1; }
  echo "on  rep$rep: $(tail -1 gpurun_out/tunable_on_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
