set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-s4}; mkdir -p $O
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/async_profile.py --consistency -1 --iters 300 > $O/async_profile.json 2> $O/async_profile.err; echo "async profile rc=$?"
for c in -1 10; do
  timeout -k 10 300 python bench.py --consistency $c --steps 300 --warmup 30 > $O/bench_c$c.json 2> $O/bench_c$c.err; echo "bench c=$c rc=$? $(python -c "import json;d=json.load(open('$O/bench_c$c.json'));print(d['value'], d['ms_per_step'])")"
done
