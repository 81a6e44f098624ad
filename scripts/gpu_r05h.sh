#!/bin/bash
# Round 5: the flat plan kernel (k_wf_deps) and the prefetching C5 UB pass --
# parity tests, the UB library A/B (C5 step), and a kernel-trace profile of the
# default bench for the plan's time.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wf_plan.py tests/test_gpu_lanczos.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest.log | head; tail -30 $O/pytest.log; exit $rc; }
AB_SCRIPT=ab_c5.py bash scripts/gpu_lib_ab.sh r05h/ub "--steps 10" cur ubold || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 $R/bench.py --steps 20 --warmup 3 > $O/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $O/prof_bench.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
head -c 300 $O/prof_bench.log
echo done
