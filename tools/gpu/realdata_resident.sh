#!/bin/bash
# Real-data training on packed shards, HBM-resident frames (data/resident.py, --data_residency hbm) vs the host-gather
# loader, 4 epochs of 24 batches each at the bench config; every epoch's samples/s is reported.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step rd_pack 300 python -u tools/pack_shards.py --src /tmp/lt_npz --dst /tmp/lt_shard --fake 100 --steps 40 --hw 360 640
rm -rf /tmp/lt_npz
for mode in hbm host; do
    TAIL=12 run_step rd_train_$mode 600 python -u distribute_train.py --dataset_dir /tmp/lt_shard --height 300 --width 300 \
        --batch_size 128 --max_epochs 4 --limit_train_batches 24 --limit_val_batches 2 --num_workers 16 \
        --log_every_n_steps 8 --log_dir /tmp/exp_logs_$mode --ckpt_dir /tmp/exp_ckpt_$mode --data_residency $mode
done
