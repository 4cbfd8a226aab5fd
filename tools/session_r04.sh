#!/bin/bash
# Round-4 GPU session: evaluation probe, tile-resident riders (tests, phase timeline, A/B bench), IPC ranks.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_s5; mkdir -p $OUT
timeout -k 10 60 ./tools/eval_probe 200 > $OUT/eval_probe.json 2> $OUT/eval_probe.err; rc=$?; echo "probe rc=$rc"; cat $OUT/eval_probe.json
[ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lanes.py::test_tile_resident_riders_rows_equal_pair_major tests/test_gpu_ipc_lanes.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 0 1; do
  PSX_RIDERS_TILE=$v PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 >> $OUT/lanes_profile.jsonl 2>> $OUT/lanes_profile.err || exit 1
done
python -c "
import json
for l in open('$OUT/lanes_profile.jsonl'):
    d=json.loads(l); print(d['us_per_round'], d.get('riders'), [p.get('solve_total') for p in d.get('phases',[])])"
for v in 0 1 0 1; do
  PSX_RIDERS_TILE=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $OUT/ab.tmp 2>> $OUT/ab.err || exit 1
  echo "[tile=$v] $(python -c "import json;d=json.load(open('$OUT/ab.tmp'));print(d['value'],d['ms_per_step'])")" | tee -a $OUT/ab.txt
done
echo done
