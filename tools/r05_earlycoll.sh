# Round 5: the multi-rank lanes loop's early collectives (PSX_EARLY_COLL) -- correctness
# (IPC rehearsals against the in-process engine) and the world-1 RCCL rehearsal's rate.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-earlycoll}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ipc_lanes.py -k "ranks_equal or stop_vote" > $O/pytest_ipc.log 2>&1; rc=$?
echo "ipc rc=$rc"; grep -E "PASS|FAIL" $O/pytest_ipc.log | head
[ $rc -eq 0 ] || exit $rc
for ec in 1 0; do
  PSX_EARLY_COLL=$ec PSX_BENCH_DIST=1 timeout -k 10 300 python bench.py --colocated-server --steps 300 --warmup 30 --no-accuracy-run > $O/dist1_ec$ec.json 2> $O/dist1_ec$ec.err; rc=$?
  echo "world-1 early=$ec rc=$rc $(python -c "
import json;t=open('$O/dist1_ec$ec.json').read();i=t.find('{\"metric\"');d=json.loads(t[i:].splitlines()[0]);print(d['value'],d['ms_per_step'])" 2>/dev/null)"
  case $rc in 124|137|134|139) exit $rc;; esac
done
