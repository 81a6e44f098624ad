#!/bin/bash
# Round 6: kernel trace of the CU-partitioned SpMM (do the tile and prefetch
# kernels overlap in time?)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r06h
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/scripts/ab_c3.py --spmm-only --rounds 1 "LZ_SPMM_PF=2,8,96" > $O/trace.log 2>&1
rc=$?; tail -3 $O/trace.log; find $O/trace -name "*.csv" | head; exit $rc
