#!/bin/bash
# Round-3 GPU session X: the comm / lanes GPU tests (incl. the CLI defaults on the
# multi-rank lanes loop), then the reference's 8-run matrix on one MI355X with the final
# round-3 engine (every BSP run on the lanes loop, cadence in the native loop; SSP/ASP
# through the in-process asynchronous scheduler), default cadence, 1,000 s per run.
set -o pipefail
OUT=gpurun_out/matrix_final
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_lanes.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest.log && exit 1
timeout -k 10 1070 python -u tools/experiment_matrix.py --device cuda --seconds 1000 --out $OUT > $OUT/matrix.out 2>&1
echo "matrix rc=$?"
