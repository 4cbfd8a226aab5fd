# Round 5: where the sparse (wide-model) configs spend their time.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-sparse}; mkdir -p $O
timeout -k 10 300 python bench.py --model sparse1m --steps 40 --warmup 10 > $O/sparse1m.json 2> $O/sparse1m.err; echo "sparse1m rc=$? $(python -c "import json;d=json.load(open('$O/sparse1m.json'));print(d['value'], d['ms_per_step'], d['config']['parallelism'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o sp -- python bench.py --model sparse1m --steps 40 --warmup 10 > $O/sparse1m_prof.json 2> $O/sparse1m_prof.err; echo "prof rc=$?"
find $O/prof -name "*kernel_stats.csv" | head -3
