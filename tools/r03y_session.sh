#!/bin/bash
# Round-3 GPU session Y: PMC passes of the default bench (8 workers per GPU) and the
# phase timeline at 8 lanes, final build.
set -o pipefail
OUT=gpurun_out/r03y
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 > $OUT/lanes_profile_w8.jsonl 2> $OUT/lanes_profile.err || exit 1
PMC_STEPS=200 bash tools/pmc_profile.sh > $OUT/pmc_passes.txt 2>&1
echo "session done"
