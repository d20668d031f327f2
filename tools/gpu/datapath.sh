#!/bin/bash
# Real-data input path on one MI355X: pack random 360x640 episodes into shards (in /tmp on the box), then run the
# training entrypoint on them at the bench config (300x300, b128, T=6) and report the trainer's samples/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-data}
EPS=${EPS:-100}
timeout -k 10 300 python -u tools/pack_shards.py --src /tmp/lt_npz --dst /tmp/lt_shard --fake $EPS --steps 40 --hw 360 640 \
  > gpurun_out/${TAG}_pack.log 2>&1 || { echo "pack failed"; tail gpurun_out/${TAG}_pack.log; exit 1; }
tail -3 gpurun_out/${TAG}_pack.log
rm -rf /tmp/lt_npz
timeout -k 10 600 python -u distribute_train.py --dataset_dir /tmp/lt_shard --height 300 --width 300 --batch_size 128 \
  --max_epochs ${EPOCHS:-2} --limit_train_batches ${BATCHES:-24} --limit_val_batches 2 --num_workers 16 --log_every_n_steps 8 \
  --log_dir /tmp/exp_logs --ckpt_dir /tmp/exp_ckpt ${TRAIN_ARGS} > gpurun_out/${TAG}_train.log 2>&1 || { echo "train failed $?"; tail -30 gpurun_out/${TAG}_train.log; exit 1; }
grep -E "^epoch|test_loss|samples" gpurun_out/${TAG}_train.log | tail -8
