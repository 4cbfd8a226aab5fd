#!/bin/bash
# Round-3 GPU session D: placement rotation check, the GPU suite, bench forms.
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python - > $OUT/xcc_rotation.txt 2>&1 <<'PY'
import torch
from psx import _native
h = _native.hip()
s = torch.cuda.current_stream().cuda_stream
for pre in [0, 1, 3, 5, 7, 9, 13]:
    if pre:
        h.xcc_map(pre, s)  # a launch with `pre` workgroups first
    m = h.xcc_map(64, s)
    off = [(m[b] - b) % 8 for b in range(64)]
    print("after a", pre, "workgroup launch: offsets", sorted(set(off)), "first 16:", m[:16])
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
for W in 1 4 7 8; do
  timeout -k 10 120 python bench.py --workers $W --steps 2000 --warmup 200 > $OUT/bench_w$W.json 2> $OUT/bench_w$W.err || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err
echo "session done"
