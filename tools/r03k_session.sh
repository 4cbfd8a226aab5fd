#!/bin/bash
# Round-3 GPU session K: persistent wide solve (tests + sharded100m bench, chain
# vs persistent), 8 workers -- riders vs side-stream evaluation with event /
# stream-value ordering; many-slot persistent dense solve test.
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_keyrange.py tests/test_gpu_kernels.py -k "keyrange or persistent_wide or pulled or many_slots or retries" -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model sharded100m > $OUT/kr_persist.json 2> $OUT/kr_persist.err || exit 1
PSX_WIDE_PERSIST=0 timeout -k 10 300 python bench.py --model sharded100m --steps 300 --warmup 30 > $OUT/kr_chain.json 2> $OUT/kr_chain.err || exit 1
for mode in riders event value; do
  if [ $mode = riders ]; then export PSX_LANES_SIDE_EVAL=0; else export PSX_LANES_SIDE_EVAL=1; export PSX_SIDE_SYNC=$mode; fi
  timeout -k 10 120 python bench.py --workers 8 --no-accuracy-run > $OUT/w8_$mode.json 2> $OUT/w8_$mode.err || exit 1
done
unset PSX_LANES_SIDE_EVAL PSX_SIDE_SYNC
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kr -- python3 bench.py --model sharded100m --steps 300 --warmup 30 > $OUT/kr_prof.json 2> $OUT/prof_kr.err || exit 1
echo "session done"
