#!/bin/bash
# Round 5: kernel-level changes -- parity tests (plan, Lanczos paths) and a
# kernel-trace profile of the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r05i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wf_plan.py tests/test_gpu_lanczos.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest.log | head; tail -30 $O/pytest.log; exit $rc; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 $R/bench.py --steps 20 --warmup 3 > $O/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $O/prof_bench.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -size +20M -delete
grep -o '"value": [0-9.]*' $O/prof_bench.log | head -1
echo done
