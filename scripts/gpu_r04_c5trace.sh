#!/bin/bash
# Kernel trace of the C5 leg alone (b = 32 fp32 power-law): the SpMM's main and long-tile passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r04c5t}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --c5-steps 10 > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/trace.log; exit 1; }
cut -c1-170 $O/trace/run_kernel_stats.csv | head -14
