#!/bin/bash
# FETCH_SIZE / WRITE_SIZE on known-byte kernels (tools/pmc_calibrate.py), one TCC counter group per pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/cal_$c -o pmc -- python3 tools/pmc_calibrate.py \
    > gpurun_out/cal_$c.log 2>&1 || { echo "pmc $c failed $?"; tail -5 gpurun_out/cal_$c.log; exit 1; }
done
find gpurun_out/cal_* -name "*.db" -delete
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"gpurun_out/cal_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                print(c, r["Kernel_Name"][:60], f"{float(r['Counter_Value']) * 1024 / 1e9:.3f} GB")
PY
tail -1 gpurun_out/cal_FETCH_SIZE.log
