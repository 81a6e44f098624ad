#!/bin/bash
# Round 5: b = 32 fp32 Gram with four units of loads in flight -- the C5 and
# b = 32 tests, then a kernel-trace profile of the bench's C5 leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05zd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py tests/test_gpu_kernels.py tests/test_gpu_vranks.py -m gpu -x -v -k "c5 or b32 or powerlaw or gram or fused_any_b or final_state" --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest.log | head; tail -30 $O/pytest.log; exit $rc; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 $R/bench.py --no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --c5-steps 10 > $O/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $O/prof_bench.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
echo done
