#!/bin/bash
# Round-5 end-of-round evidence on the committed sources: the -m gpu suite,
# smoke(), the default bench line (with the r05 counter files now matching the
# launched kernels), the c4rank line and a kernel-trace profile of the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r05g}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 python -u bench.py --config c4rank > $O/bench_c4rank.json 2> $O/bench_c4rank.err || { echo "c4rank failed"; tail -20 $O/bench_c4rank.err; exit 1; }
cut -c1-300 $O/bench_c4rank.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 $R/bench.py --steps 20 --warmup 3 > $O/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $O/prof_bench.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -2
find $O/prof -name "*kernel_trace.csv" -size +30M -delete
echo done
