#!/bin/bash
# se_rowmat (16-frame tiles, V prefetched, no per-element division) + adaptive se_wsum_part slices: numerics, isolated
# A/B vs the committed HEAD build, bench A/B; default-priority comm stream check; real-data training with the
# training stream at high vs default priority.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/head2/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step se_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_backbone_gpu.py \
    tests/test_pwgemm_gpu.py -k "se_ or pw_z"
run_step se_ab2 300 python -u tools/bench_se.py --ab $BASE_SO
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step se_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step se_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
RT1_DP_DIAG=comminit TAIL=1 run_step dm_comminit 300 python -u bench.py --steps 20 --warmup 5
run_step rd_pack 300 python -u tools/pack_shards.py --src /tmp/lt_npz --dst /tmp/lt_shard --fake 100 --steps 40 --hw 360 640
for mode in high normal high normal; do
  RT1_TRAIN_STREAM=$mode TAIL=12 run_step rd_train_$mode 600 python -u distribute_train.py --dataset_dir /tmp/lt_shard \
      --height 300 --width 300 --batch_size 128 --max_epochs 3 --limit_train_batches 24 --limit_val_batches 2 \
      --num_workers 16 --log_every_n_steps 24 --log_dir /tmp/exp_logs_$mode --ckpt_dir /tmp/exp_ckpt_$mode \
      --data_residency hbm
done
