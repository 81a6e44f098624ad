#!/bin/bash
# End-of-milestone GPU evidence, part 1: tests, smoke, the default bench line
# (+ CPU baseline and parity), the N > 1 code path rehearsed at N = 1 (both
# exchange forms), the single-GPU C4 line.
#   bash scripts/gpu_round.sh TAG        (part 2: scripts/gpu_round_prof.sh TAG)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --dist --no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0 --spmm-reps 0 > $O/dist_halo.json 2> $O/dist_halo.err || { tail -20 $O/dist_halo.err; exit 1; }
timeout -k 10 300 python bench.py --dist --exchange allgather --no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0 --spmm-reps 0 > $O/dist_allgather.json 2> $O/dist_allgather.err || { tail -20 $O/dist_allgather.err; exit 1; }
timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 2 --spmm-reps 5 > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
echo done
