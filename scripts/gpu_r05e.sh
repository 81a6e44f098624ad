#!/bin/bash
# Round 5: the column-panel SpMM candidate -- parity tests, the A/B against
# k_spmm_seg at C3, then FETCH / WRITE and the texture-path counter groups of both.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v -k "panel" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_panel.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/pytest_panel.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_panel.log | tail -8
timeout -k 10 400 python -u scripts/panel_ab.py --rounds 5 > $O/panel_ab.log 2>&1 || { echo "ab rc=$?"; tail -20 $O/panel_ab.log; exit 1; }
grep -v amdgpu.ids $O/panel_ab.log | tail -7
