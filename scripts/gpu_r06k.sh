#!/bin/bash
# Round 6: the CU-partitioned SpMM with shader-engine-balanced masks.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 300 python -u scripts/ab_c3.py --spmm-only --rounds 2 "LZ_SPMM_PF=0" "LZ_SPMM_PF=0,0" "LZ_SPMM_PF=1,0" \
  "LZ_SPMM_PF=2,0" "LZ_SPMM_PF=1,8,96" "LZ_SPMM_PF=2,8,96" "LZ_SPMM_PF=1,8,32" "LZ_SPMM_PF=2,16,96" "LZ_SPMM_PF=1,4,192" \
  > $O/pf_ab.log 2>&1
rc=$?; grep round $O/pf_ab.log; exit $rc
