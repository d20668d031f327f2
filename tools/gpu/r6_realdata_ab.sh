#!/bin/bash
# Real-data resident training: step stream at high priority (default) vs RT1_TRAIN_STREAM=normal, same box, + bench
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step rd2_bench 400 python -u bench.py --steps 20 --warmup 5
run_step rd2_pack 300 python -u tools/pack_shards.py --src /tmp/lt_npz --dst /tmp/lt_shard --fake 100 --steps 40 --hw 360 640
rm -rf /tmp/lt_npz
for st in normal high; do
    RT1_TRAIN_STREAM=$st TAIL=12 run_step rd2_train_$st 500 python -u distribute_train.py --dataset_dir /tmp/lt_shard --height 300 --width 300 \
        --batch_size 128 --max_epochs 3 --limit_train_batches 24 --limit_val_batches 2 --num_workers 16 \
        --log_every_n_steps 8 --log_dir /tmp/exp_logs_$st --ckpt_dir /tmp/exp_ckpt_$st --data_residency hbm
done
