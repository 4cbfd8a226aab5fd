set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-sparse2}; mkdir -p $O
for w in 4 8; do
  timeout -k 10 300 python bench.py --model sparse1m --workers $w --steps 40 --warmup 10 > $O/sparse1m_w$w.json 2> $O/sparse1m_w$w.err; rc=$?
  echo "sparse1m w$w rc=$rc $(python -c "import json;d=json.load(open('$O/sparse1m_w$w.json'));print(d['value'], d['ms_per_step'], d['config']['parallelism'])" 2>/dev/null)"; tail -2 $O/sparse1m_w$w.err | cut -c1-300
  case $rc in 124|137|134|139) exit $rc;; esac
done
timeout -k 10 300 python bench.py --model sharded100m --steps 40 --warmup 10 > $O/sharded100m.json 2> $O/sharded100m.err; echo "sharded100m rc=$? $(python -c "import json;d=json.load(open('$O/sharded100m.json'));print(d['value'], d['ms_per_step'], d['config']['parallelism'])" 2>/dev/null)"
