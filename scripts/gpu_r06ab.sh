#!/bin/bash
# Round 6: pass UB's overlap -- the diagnostic build with its MFMAs skipped (LZ_UB_DMA=33) or its
# DMAs, waits and stores skipped (65) against the full pass (1); results wrong in the two diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
export LZ_HIP_LIB=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib/liblz_hip_diag.so
timeout -k 10 400 python -u scripts/ab_c5.py "LZ_UB_DMA=1" "LZ_UB_DMA=33 AB_NOCHECK=1" "LZ_UB_DMA=65 AB_NOCHECK=1" --rounds 3 > $O/ub_overlap.log 2>&1 || { tail -20 $O/ub_overlap.log; exit 1; }
grep round $O/ub_overlap.log
