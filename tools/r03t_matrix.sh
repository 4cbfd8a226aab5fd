#!/bin/bash
# Round-3 GPU session T: the reference's 8-run matrix on one MI355X with the
# disjoint-window cadence (--iter_new_frac 1.0 --iter_new_cap 256: a worker iterates
# once its whole window is new), 1,040 s per run, all 8 engines side by side.
set -o pipefail
OUT=gpurun_out/matrix_f100
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1150 python -u tools/experiment_matrix.py --device cuda --seconds 1040 --iter_new_frac 1.0 --iter_new_cap 256 --out $OUT > $OUT/matrix.out 2>&1
echo "matrix rc=$?"
