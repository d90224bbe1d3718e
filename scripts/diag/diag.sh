set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=temporal_inverse_kinematics_amd
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -fPIC -std=c++17 -Iinclude"
$H -c $P/csrc/misc.hip -o /tmp/misc.o && $H -x hip -c $P/csrc/api.cpp -o /tmp/api.o && $H -c $P/csrc/cgemm.hip -o /tmp/cg.o && $H -shared -o /tmp/libtik_a.so /tmp/misc.o /tmp/api.o /tmp/cg.o || exit 2
$H -mcode-object-version=5 -c $P/csrc/misc.hip -o /tmp/misc5.o && $H -mcode-object-version=5 -x hip -c $P/csrc/api.cpp -o /tmp/api5.o && $H -mcode-object-version=5 -c $P/csrc/cgemm.hip -o /tmp/cg5.o && $H -mcode-object-version=5 -shared -o /tmp/libtik_5.so /tmp/misc5.o /tmp/api5.o /tmp/cg5.o || exit 2
$H scripts/diag/launch_test.cpp -L/tmp -l:libtik_a.so -Wl,-rpath,/tmp -o /tmp/launch_test || exit 2
echo "== standalone (rocm 7.2 runtime)"; timeout -k 5 60 /tmp/launch_test; echo rc=$?
echo "== torch + default lib"; timeout -k 5 120 python scripts/diag/diag.py torch /tmp/libtik_a.so; echo rc=$?
echo "== torch + cov5 lib"; timeout -k 5 120 python scripts/diag/diag.py torch /tmp/libtik_5.so; echo rc=$?
ls -la /usr/local/lib/python3.10/dist-packages/torch/lib/libamdhip64.so /opt/rocm/lib/libamdhip64.so*
exit 0
