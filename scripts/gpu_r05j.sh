#!/bin/bash
# Round 5: the N = 1 RCCL rehearsals of the distributed path (halo and
# all-gather forms) through torchrun, as the driver launches N > 1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
for ex in halo allgather; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --exchange $ex --no-cpu-baseline > $O/dist_$ex.json 2> $O/dist_$ex.err || { echo "dist $ex failed rc=$?"; tail -20 $O/dist_$ex.err; exit 1; }
  cut -c1-300 $O/dist_$ex.json
done
