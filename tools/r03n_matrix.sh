#!/bin/bash
# Round-3 GPU session N: phase timeline of the lanes kernel (4 and 8 lanes, with the
# per-slot sub-phases), then the two producer-clock runs of the reference matrix that
# faulted on the Python concurrent-stream path (4 workers at 0.5 and 5 tps), now on
# the lanes loop with the cadence in the native loop; both engines on one MI355X.
set -o pipefail
OUT=gpurun_out/matrix_gpu2
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for L in 4 8; do
  PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl 2> $OUT/lanes_profile.err || exit 1
done
timeout -k 10 1080 python -u tools/experiment_matrix.py --device cuda --seconds 1000 --runs 4-workers_0-5tps,4-workers_5tps --out $OUT > $OUT/matrix.out 2>&1
echo "matrix rc=$?"
