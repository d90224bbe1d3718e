# Same-box A/B: the in-tree libtik.so vs ab/libtik_base.so (scripts/build_base.sh),
# alternating, $1 rounds (default 2). Prints value, ms/step and the per-launch times.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ablib; mkdir -p $O
N=${1:-2}
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { tail -20 $O/pt.log; exit 1; }
  tail -1 $O/pt.log
fi
for r in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then export TIK_LIB=ab/libtik_base.so; else unset TIK_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/$v$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/$v$r.json'));l=d['forward']['launches'];print('$v', d['value'], d['ms_per_step'], ' '.join(f'{k.split(\".\")[-1]}={v[\"avg_ms\"]}' for k,v in l.items()))"
  done
done
