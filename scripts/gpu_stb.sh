# persistent stblock: GPU tests, phase trace, A/B against one workgroup per tile
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { tail -20 $O/pt.log; exit 1; }
tail -2 $O/pt.log
TIK_SPLIT=0 TIK_STB_TRACE=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compare --no-profile > $O/tr.json 2> $O/tr.err || exit 1
grep stblock $O/tr.err | tail -2
for r in 1 2; do
  for e in ""; do
    if [ -n "$e" ]; then export TIK_STB_ONE_TILE=1; else unset TIK_STB_ONE_TILE; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare > $O/r$r$e.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/r$r$e.json'));l=d['forward']['launches'];print('one_tile=$e', d['value'], d['ms_per_step'], l['B0_64.L0']['avg_ms'], l['B3_64.L1']['avg_ms'])"
  done
done
