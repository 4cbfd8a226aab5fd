#!/bin/bash
# Round-3 GPU session S: cadence pilot on the reference's 4 workers x 10 tps run
# (psx trails there at 300 s): three cadences side by side on one MI355X, 330 s each.
set -o pipefail
OUT=gpurun_out/cadence
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import sys; sys.path[:0] = ['tools', '.']; import experiment_matrix as m; m.ensure_data('data')" > $OUT/data.log 2>&1 || exit 1
run() {  # name frac cap
  timeout -k 10 400 python -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin \
    -p 25 -c 0 --num_workers 4 -l --log_dir $OUT/$1 --max_wallclock_s 330 --async_scheduler threads \
    --iter_new_frac $2 --iter_new_cap $3 > $OUT/$1.out 2>&1
  echo "$1 rc=$?" >> $OUT/rc.txt
}
run f50c128 0.5 128 &
run f25c128 0.25 128 &
run f50c48 0.5 48 &
run f100c256 1.0 256 &
while [ $(jobs -r | wc -l) -gt 0 ]; do sleep 20; echo "$(date +%s) running $(jobs -r | wc -l)" >> $OUT/progress.txt; done
wait
cat $OUT/rc.txt
