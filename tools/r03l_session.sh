#!/bin/bash
# Round-3 GPU session L (re-entry): GPU suite + smoke + the driver's bench forms,
# the 4-worker producer-clock matrix config for 40 s on the lanes loop (cadence in
# the native loop), then the same on the Python concurrent-stream path (the fault).
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest_gpu.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || exit 1
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import sys; sys.path[:0] = ['tools', '.']; import experiment_matrix as m; m.ensure_data('data')" > $OUT/data.log 2>&1 || exit 1
timeout -k 10 120 python -X faulthandler -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin -p 500 -c 0 --num_workers 4 -l --log_dir $OUT/run_lanes --max_wallclock_s 40 --async_scheduler threads > $OUT/run_lanes.out 2>&1 || exit 1
PSX_NATIVE_LANES=0 timeout -k 10 120 python -X faulthandler -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin -p 500 -c 0 --num_workers 4 -l --log_dir $OUT/run_py --max_wallclock_s 40 --async_scheduler threads > $OUT/run_py.out 2>&1
echo "rc=$?" >> $OUT/run_py.out
echo "session done"
