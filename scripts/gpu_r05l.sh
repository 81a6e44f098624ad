#!/bin/bash
# Round 5: the full-size C5 parity test.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py -m gpu -x -v -k "c5_full_size or final_state or powerlaw" --timeout 400 --timeout-method thread -p no:cacheprovider --durations=5 > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest.log | head; tail -30 $O/pytest.log; exit $rc; }
grep -A7 "slowest" $O/pytest.log
