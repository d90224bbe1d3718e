#!/bin/bash
# Copy a GPU session's summaries from gpurun_out/ (scratch) into profiles/ (tracked)
# as profiles/<round>_<tag>_*. Usage: bash scripts/save_profiles.sh TAG ROUND   (e.g. r05a r05_a)
set -u
TAG=$1; P=profiles/$2; O=gpurun_out
cp_if() { [ -f "$1" ] && cp "$1" "$2"; }
cp_if $O/pmc_traffic_$TAG.json ${P}_pmc_traffic.json
cp_if $O/pmc_traffic_$TAG.txt ${P}_pmc_traffic.txt
cp_if $O/pmc_mfma_$TAG.json ${P}_pmc_mfma.json
cp_if $O/pmc_mfma_$TAG.txt ${P}_pmc_mfma.txt
cp_if $O/bench_$TAG.json ${P}_bench.json
cp_if $O/fk_$TAG.json ${P}_bench_fk.json
cp_if $O/stream_$TAG.json ${P}_stream_online.json
cp_if $O/train_$TAG.json ${P}_bench_train.json
cp_if $O/pytest_gpu_$TAG.log ${P}_pytest_gpu.log
cp_if $O/smoke_$TAG.log ${P}_smoke.log
f=$(find $O/prof_$TAG -name '*kernel_stats.csv' 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" ${P}_kernel_stats.csv
ls -la ${P}_* 2>/dev/null
