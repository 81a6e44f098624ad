#!/bin/bash
# Round 5: the distributed wavefront solve with beta_0's Gram from the first
# launch -- virtual-rank and distributed tests, then the N = 1 RCCL rehearsals.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05ze
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_vranks.py tests/test_gpu_dist.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest.log | head; tail -30 $O/pytest.log; exit $rc; }
for ex in halo allgather; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --exchange $ex --no-cpu-baseline > $O/dist_$ex.json 2> $O/dist_$ex.err || { echo "dist $ex failed rc=$?"; tail -20 $O/dist_$ex.err; exit 1; }
  cut -c1-200 $O/dist_$ex.json
done
