#!/bin/bash
# Round 6: kernel trace of the C5 leg (main tile pass vs the long-tile pass beside it).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
O=$ROOT/gpurun_out/r06v
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- python3 $ROOT/bench.py \
  --no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --c5-steps 10 > $O/trace_c5.log 2>&1 || { tail -5 $O/trace_c5.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -2
