set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/wide_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model sparse1m > gpurun_out/bench_sparse1m.log 2>&1
rc=$?; tail -1 gpurun_out/bench_sparse1m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model sharded100m > gpurun_out/bench_sharded100m.log 2>&1
rc=$?; tail -1 gpurun_out/bench_sharded100m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sparse -o run -- python3 bench.py --model sparse1m --steps 100 --warmup 10 > gpurun_out/prof_sparse.log 2>&1
rc=$?; echo prof rc=$rc; exit $rc
