set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s2; mkdir -p $O
PYT="python -u -m pytest -v -s --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT -x tests/test_gpu_ipc_lanes.py -k peer > $O/pytest_peer.log 2>&1; rc=$?
echo "peer rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_peer.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 $PYT tests/test_gpu_async_lanes.py tests/test_gpu_ipc_lanes.py -k "not peer" > $O/pytest_async.log 2>&1; rc=$?
echo "async rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|replay c=" $O/pytest_async.log | tail -20
[ $rc -le 1 ] || exit $rc
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 > $O/lanes_profile.jsonl 2> $O/lanes_profile.err; echo "timeline rc=$?"
