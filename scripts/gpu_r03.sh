#!/bin/bash
# Round-3 evidence run: the GPU suite, the default bench (every leg checked
# against the oracle), the N>1 code path rehearsed at N = 1 (both exchanges),
# smoke.  Usage: scripts/gpu_r03.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|ERROR" $O/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_dist_halo.json 2> $O/bench_dist_halo.err || { tail $O/bench_dist_halo.err; exit 1; }
timeout -k 10 300 python bench.py --dist --exchange allgather --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_dist_ag.json 2> $O/bench_dist_ag.err || { tail $O/bench_dist_ag.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
