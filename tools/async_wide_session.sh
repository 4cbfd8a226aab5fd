#!/bin/bash
# Wide (sparse) model with N in-process ASP workers: event scheduler vs threads; kernel stats of the
# dense 8-worker ASP run under the event scheduler.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/async_wide
mkdir -p $OUT
for n in 2 4; do
  for s in events threads; do
    timeout -k 10 240 python bench.py --model sparse1m --workers $n --steps 200 --warmup 20 --async-scheduler $s > $OUT/sp_w${n}_$s.log 2>&1
    rc=$?
    python -c "import json; d=[json.loads(l) for l in open('$OUT/sp_w${n}_$s.log') if l.startswith('{')][-1]; print('sparse1m w=$n $s', d['value'], d['ms_per_step'], d['best_test_f1'])" || true
    [ $rc -eq 0 ] || { tail -20 $OUT/sp_w${n}_$s.log; exit $rc; }
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workers 8 --consistency -1 --steps 300 --warmup 30 > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '^{' $OUT/prof.log | cut -c1-200
echo async_wide done
