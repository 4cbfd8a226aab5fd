# Round 5: solver numerics + the BSP / async timelines and benches of the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-perf}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lanes.py tests/test_gpu_async_lanes.py tests/test_gpu_engine.py > $O/pytest_lanes.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_lanes.log; grep -E "FAILED|ERROR" $O/pytest_lanes.log | head
[ $rc -eq 0 ] || exit $rc
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 > $O/lanes_profile.jsonl 2> $O/lanes_profile.err; echo "timeline rc=$?"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_short.json 2> $O/bench_short.err; echo "bench short rc=$? $(python -c "import json;d=json.load(open('$O/bench_short.json'));print(d['value'], d['ms_per_step'])")"
SESS=${SESS:-perf} bash tools/r05_s4.sh
