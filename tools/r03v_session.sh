#!/bin/bash
# Round-3 GPU session V: the evaluation as a launch of its own right behind each round
# (PSX_SIDE_SYNC=inline; more, smaller workgroups than the riders) against the riders,
# at 4 and 8 lanes; its rows against the riders' rows.
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PSX_SIDE_SYNC=inline timeout -k 10 200 python -u -m pytest tests/test_gpu_lanes.py -k side_stream -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
for L in 4 8; do
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 | sed "s/^/riders /" >> $OUT/profile.txt || exit 1
  for G in 256 512 1024; do
    PSX_LANES_SIDE_EVAL=1 PSX_SIDE_SYNC=inline PSX_SIDE_GRID=$G timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 | sed "s/^/inline$G /" >> $OUT/profile.txt || exit 1
  done
  PSX_LANES_SIDE_EVAL=1 timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 | sed "s/^/corun256 /" >> $OUT/profile.txt || exit 1
done
echo "session done"
