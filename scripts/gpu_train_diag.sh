#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 120 python tests/diag/train_diff.py 8 9 golden 2>&1 | grep "<<<\|loss\|^L\|^B\|Error"
