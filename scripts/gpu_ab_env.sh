# A/B of one env hook on the IK bench: bash scripts/gpu_ab_env.sh VAR  (runs VAR unset, VAR=1, twice each)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V=$1; VAL=${2:-1}
O=gpurun_out/ab_$V; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 120 --timeout-method thread -k "tgw or gpw or golden" > $O/pt.log 2>&1 || { tail -5 $O/pt.log; exit 1; }
for r in 1 2; do
  for e in "" $VAL; do
    if [ -n "$e" ]; then export $V=$e; else unset $V; fi; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/r$r$e.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/r$r$e.json'));l=d['forward']['launches'];print('$V=$e', d['value'], d['ms_per_step'], l.get('TW_128.L3',{}).get('avg_ms'), l.get('TW_128.L4',{}).get('avg_ms'))"
  done
done
