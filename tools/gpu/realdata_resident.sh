#!/bin/bash
# Real-data training on packed shards, HBM-resident frames (data/resident.py, --data_residency hbm) against the same
# box's synthetic bench: bench.py first, then 4 epochs of 24 batches at the bench config; every epoch's samples/s is
# reported.  MODES="hbm host" also runs the host-gather loader.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step rd_bench 400 python -u bench.py --steps 20 --warmup 5
run_step rd_pack 300 python -u tools/pack_shards.py --src /tmp/lt_npz --dst /tmp/lt_shard --fake 100 --steps 40 --hw 360 640
rm -rf /tmp/lt_npz
for mode in ${MODES:-hbm}; do
    TAIL=30 run_step rd_train_$mode 600 python -u distribute_train.py --dataset_dir /tmp/lt_shard --height 300 --width 300 \
        --batch_size 128 --max_epochs ${EPOCHS:-4} --limit_train_batches ${BATCHES:-24} --limit_val_batches 2 --num_workers 16 \
        --log_every_n_steps 8 --log_dir /tmp/exp_logs_$mode --ckpt_dir /tmp/exp_ckpt_$mode --data_residency $mode
done
