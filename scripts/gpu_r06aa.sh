#!/bin/bash
# Round 6: the N-rank launcher end to end on a one-GPU box: --gpus 2 starts two ranks
# under torch.distributed.run; rank 1 has no device, so the run must fail, non-zero, with no JSON line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 180 python bench.py --gpus 2 --steps 2 --warmup 1 > $O/launch2.out 2> $O/launch2.err
echo "rc=$?"
wc -c < $O/launch2.out
grep -E "starting 2 ranks|invalid device|ChildFailedError|Error" $O/launch2.err | head -8
exit 0
