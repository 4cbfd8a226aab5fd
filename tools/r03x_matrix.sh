#!/bin/bash
# Round-3 GPU session X: the reference's 8-run matrix on one MI355X with the final
# round-3 engine (every BSP run on the lanes loop, cadence in the native loop; SSP/ASP
# through the in-process asynchronous scheduler), default cadence, 1,040 s per run.
set -o pipefail
OUT=gpurun_out/matrix_final
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1150 python -u tools/experiment_matrix.py --device cuda --seconds 1040 --out $OUT > $OUT/matrix.out 2>&1
echo "matrix rc=$?"
