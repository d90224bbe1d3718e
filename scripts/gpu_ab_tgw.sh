# A/B of the weight-stationary kernel against TG3 on the same box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab; mkdir -p $O; TAG=${1:-x}
for v in 1 0 1 0; do
  TIK_TGW=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare > $O/b_${TAG}_$v.json 2> $O/b_${TAG}_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/b_${TAG}_$v.json'));L=d['forward']['launches'];print('TGW=$v', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in L.items() if 'L3' in k or 'L4' in k})"
done
TIK_TG_TRACE=1 timeout -k 10 100 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compare > /dev/null 2> $O/trace_$TAG.err || exit $?
grep "TW L" $O/trace_$TAG.err | tail -2
