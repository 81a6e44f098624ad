#!/bin/bash
# Distributed entry points on one GPU: tests, then the bench's N>1 code path
# rehearsed at N = 1 (halo and all-gather exchanges).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/dist
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -12 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_halo.json 2> $O/bench_halo.err || { tail $O/bench_halo.err; exit 1; }
cat $O/bench_halo.json
timeout -k 10 300 python bench.py --dist --exchange allgather --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_ag.json 2> $O/bench_ag.err || { tail $O/bench_ag.err; exit 1; }
cat $O/bench_ag.json
