set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stag; mkdir -p $O
for st in 0 700 1500 0; do
  TIK_STAGGER=$st timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > $O/b$st.json 2> $O/b.err || exit $?
  python -c "import json;d=json.load(open('$O/b$st.json'));print($st, d['value'],d['ms_per_step'],{k:v['avg_ms'] for k,v in d['forward']['launches'].items() if k.startswith('T')})"
done
