#!/bin/bash
# MFMA post-call state pass: final-state tests, then the C3 A/B against the LDS form.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04y}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lanczos.py -k "final_state" > $O/fs_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/fs_tests.log; exit 1; }
tail -2 $O/fs_tests.log
timeout -k 10 300 python -u scripts/ab_c3.py "LZ_FS_MFMA=1" "LZ_FS_MFMA=0" "AB_FS=0" --rounds 4 --steps 20 > $O/fs_ab.log 2>&1 || { echo "ab failed rc=$?"; tail -5 $O/fs_ab.log; exit 1; }
grep "^round" $O/fs_ab.log
