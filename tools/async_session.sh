#!/bin/bash
# In-process SSP/ASP: event-polling scheduler vs thread-per-worker, 4 and 8 workers on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/async
mkdir -p $OUT
timeout -k 10 240 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 4 8; do
  for c in -1 3; do
    for s in events threads; do
      timeout -k 10 180 python bench.py --workers $n --consistency $c --steps 500 --warmup 50 --async-scheduler $s > $OUT/w${n}_c${c}_$s.log 2>&1
      rc=$?
      python -c "import json; d=[json.loads(l) for l in open('$OUT/w${n}_c${c}_$s.log') if l.startswith('{')][-1]; print('w=$n c=$c $s', d['value'], d['ms_per_step'], d.get('max_vc_gap'), d['best_test_f1'])" || true
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
echo async done
