set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-sparse3}; mkdir -p $O
val() { python - "$1" <<'PY'
import json,sys
t=open(sys.argv[1]).read(); i=t.find('{"metric"')
d=json.loads(t[i:].splitlines()[0]) if i>=0 else {}
print(d.get('value'), d.get('ms_per_step'))
PY
}
for se in 0 1; do
  PSX_SIDE_EVAL=$se timeout -k 10 300 python bench.py --model sparse1m --steps 40 --warmup 10 > $O/sp_se$se.json 2> $O/sp_se$se.err; rc=$?; echo "sparse1m side=$se rc=$rc $(val $O/sp_se$se.json)"
  case $rc in 124|137|134|139) exit $rc;; esac
  PSX_SIDE_EVAL=$se timeout -k 10 300 python bench.py --model sharded100m --steps 40 --warmup 10 > $O/sh_se$se.json 2> $O/sh_se$se.err; rc=$?; echo "sharded100m side=$se rc=$rc $(val $O/sh_se$se.json)"
  case $rc in 124|137|134|139) exit $rc;; esac
done
