#!/bin/bash
# Round-3 GPU session G: lanes (epoch wrap), wide (window table), key-range
# tests; default bench; sharded100m through the key-range engine.
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_wide.py tests/test_gpu_keyrange.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 python bench.py --model sharded100m > $OUT/bench_sharded100m.json 2> $OUT/bench_sharded100m.err || exit 1
echo "session done"
