#!/bin/bash
# Round-3 GPU session B: lanes kernel phase timeline + kernel trace.
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PSX_LANES_STAMPS=1
for L in 1 4 8; do
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl || exit 1
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 --no-eval >> $OUT/lanes_profile.jsonl || exit 1
done
unset PSX_LANES_STAMPS
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o w4 -- python bench.py --workers 4 --steps 200 --warmup 20 > $OUT/bench_w4_prof.json 2> $OUT/prof.err
echo "session rc=$?"
