#!/bin/bash
# Round 6: pass UB's wait for strip s with strip s-1's four row stores still in flight
# (LZ_UB_DMA=17: vmcnt(12)) against the default vmcnt(8); the bitwise test under both.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_UB_DMA=1" "LZ_UB_DMA=17" --rounds 4 > $O/ub_wait_ab.log 2>&1 || { tail -20 $O/ub_wait_ab.log; exit 1; }
grep round $O/ub_wait_ab.log
