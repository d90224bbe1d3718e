# IK step time vs DMA sub-batch size (MALL residency of the inter-layer activations)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/chunks; mkdir -p $O
for c in 0 512 256 128; do
  for sp in 1 0; do
    TIK_DMA_CHUNK=$c TIK_SPLIT=$sp timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare --steps 20 > $O/c${c}_s${sp}.json 2> $O/c${c}_s${sp}.err || exit $?
    python -c "import json;d=json.load(open('$O/c${c}_s${sp}.json'));print('chunk=$c split=$sp', d['value'], d['ms_per_step'], d.get('profiled_ms_per_step'))"
  done
done
