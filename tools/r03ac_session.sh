#!/bin/bash
# Round-3 GPU session AC: the riders publish only the K x K confusion cells to host
# memory: lanes / comm / engine tests, timeline at 4 / 8 lanes, bench forms.
set -o pipefail
OUT=gpurun_out/r03ac
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_comm.py tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest.log && exit 1
for L in 4 8; do
  PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl 2> $OUT/lanes_profile.err || exit 1
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile_nostamps.jsonl 2>> $OUT/lanes_profile.err || exit 1
done
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || exit 1
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo "session done"
