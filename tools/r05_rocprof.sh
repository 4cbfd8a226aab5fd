# Round 5: rocprofv3 kernel statistics of the BSP and ASP benches (one MI355X).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-rocprof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bsp -o bsp -- python bench.py --steps 300 --warmup 30 --no-accuracy-run > $O/bsp.json 2> $O/bsp.err; echo "bsp rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/asp -o asp -- python bench.py --consistency -1 --steps 300 --warmup 30 --no-accuracy-run > $O/asp.json 2> $O/asp.err; echo "asp rc=$?"
find $O -name "*.db" | head
