#!/bin/bash
# pass 1 with 16-bit columns: GPU tests of the touched paths, then an in-process A/B at C3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/c16
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py tests/test_gpu_vranks.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|ERROR" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_c3.py "LZ_PASS1_C16=0" "LZ_PASS1_C16=1" --rounds 5 --steps 20 > $O/ab.log 2>&1
rc=$?; tail -16 $O/ab.log; exit $rc
