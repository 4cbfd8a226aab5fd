#!/bin/bash
# Round-3 GPU session M: the four failures of session L after the fixes (persistent
# wide solve's dot partials, test assumptions), key-range suite, 8 workers with
# riders vs side-stream evaluation, sharded100m persistent vs chain.
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_keyrange.py tests/test_gpu_kernels.py tests/test_gpu_lanes.py tests/test_gpu_comm.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest.log && exit 1
for mode in riders event value; do
  if [ $mode = riders ]; then export PSX_LANES_SIDE_EVAL=0; else export PSX_LANES_SIDE_EVAL=1; export PSX_SIDE_SYNC=$mode; fi
  timeout -k 10 120 python bench.py --workers 8 --no-accuracy-run > $OUT/w8_$mode.json 2> $OUT/w8_$mode.err || exit 1
done
unset PSX_LANES_SIDE_EVAL PSX_SIDE_SYNC
timeout -k 10 300 python bench.py --model sharded100m > $OUT/kr_persist.json 2> $OUT/kr_persist.err || exit 1
PSX_WIDE_PERSIST=0 timeout -k 10 300 python bench.py --model sharded100m > $OUT/kr_chain.json 2> $OUT/kr_chain.err || exit 1
echo "session done"
