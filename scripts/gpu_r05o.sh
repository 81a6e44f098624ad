#!/bin/bash
# Round 5: non-temporal W_{j-1} loads in the C5 SpMM epilogue -- library A/B
# on the C5 step (cur: nt loads; epiplain: plain loads).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05o
AB_SCRIPT=ab_c5.py bash scripts/gpu_lib_ab.sh r05o/ab "--steps 10" cur epiplain || exit 1
