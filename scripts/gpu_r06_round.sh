#!/bin/bash
# Round-6 evidence on the current sources: the GPU suite, smoke, the default
# bench line, the N = 1 rehearsals of both exchange forms, the C4 per-rank share.
#   bash scripts/gpu_r06_round.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python bench.py --config c4rank --no-cpu-baseline > $O/bench_c4rank.json 2> $O/bench_c4rank.err || { tail -20 $O/bench_c4rank.err; exit 1; }
timeout -k 10 200 python bench.py --dist --no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0 --spmm-reps 0 > $O/bench_dist_halo.json 2> $O/bench_dist_halo.err || { tail -20 $O/bench_dist_halo.err; exit 1; }
timeout -k 10 200 python bench.py --dist --exchange allgather --no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0 --spmm-reps 0 > $O/bench_dist_allgather.json 2> $O/bench_dist_allgather.err || { tail -20 $O/bench_dist_allgather.err; exit 1; }
echo done
