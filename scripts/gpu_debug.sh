set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m temporal_inverse_kinematics_amd._build > /dev/null || exit 2
timeout -k 10 300 python tests/diag/debug_layers.py; rc=$?; echo rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q 2>&1 | tail -15
