set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/race5; mkdir -p $O
timeout -k 10 90 ./build/race_check Z 0 1500 9 > $O/z.txt 2>&1 &
vp=$!
sleep 1
pids=""
for k in 1 2 3; do AGG_SECONDS=40 timeout -k 10 80 python scripts/diag_mproc.py child > $O/aggp$k.txt 2>&1 & pids="$pids $!"; done
wait $vp
for p in $pids; do wait $p; done
grep -v "    D" $O/z.txt; grep -c "    D" $O/z.txt
echo "aggressor full-forward worst: $(cat $O/aggp*.txt | grep -v amdgpu | tr '\n' ' ')"
