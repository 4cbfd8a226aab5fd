#!/bin/bash
# In-process workers, one XCD each (persistent solves side by side): GPU suite + bench variants.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02v5_workers}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
while IFS= read -r v; do
  [ -z "$v" ] && continue
  timeout -k 10 150 python bench.py --steps 1000 --warmup 100 $v > $OUT/b.json 2>> $OUT/bench_err.log
  rc=$?; echo "bench [$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); d['variant']='$v'; print(json.dumps(d))" >> $OUT/bench_variants.jsonl
  python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('   ', d['value'], d['ms_per_step'], d['best_test_f1'])"
done <<'VARS'
--workers 4 --consistency 3
--workers 4
--workers 8
--workers 2 --consistency -1
--workers 4 --consistency -1
--workers 8 --consistency -1
VARS
echo "session done"
