#!/bin/bash
# Q-only post-call state kernel: final-state tests, C5 cost of the pass (on / off), kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r04fq}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lanczos.py -k "final_state" > $O/fs_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/fs_tests.log; exit 1; }
tail -1 $O/fs_tests.log
timeout -k 10 600 python -u scripts/ab_c5.py AB_FS=1 AB_FS=0 --rounds 3 > $O/c5_fs_ab.log 2>&1 || { echo "ab failed"; tail -5 $O/c5_fs_ab.log; exit 1; }
grep "^round" $O/c5_fs_ab.log
