#!/bin/bash
# Round-3 GPU session I: the reference's 8-run matrix at matched producer rates
# through the GPU engine (8 in-process engines on one MI355X, run concurrently).
set -o pipefail
OUT=gpurun_out/matrix_gpu
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1150 python -u tools/experiment_matrix.py --device cuda --seconds 1040 --out $OUT > $OUT/matrix.out 2>&1
echo "matrix rc=$?"
