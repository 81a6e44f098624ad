#!/bin/bash
# Round 6: the CU-partitioned SpMM A/B at C3 (DMA-streaming prefetcher; C = 0:
# the tile kernel alone on its CUs) and pass UB's store policy.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06i}
mkdir -p $O
timeout -k 10 300 python -u scripts/ab_c3.py --spmm-only --rounds 2 \
  "LZ_SPMM_PF=0" "LZ_SPMM_PF=2,0" "LZ_SPMM_PF=1,0" "LZ_SPMM_PF=2,8,96" "LZ_SPMM_PF=1,8,96" "LZ_SPMM_PF=2,16,192" \
  "LZ_SPMM_PF=3,8,96" "LZ_SPMM_PF=2,4,48" > $O/pf_ab.log 2>&1 || { tail -20 $O/pf_ab.log; exit 1; }
grep round $O/pf_ab.log
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_UB_DMA=1" "LZ_UB_DMA=5" --rounds 3 > $O/ub_ab.log 2>&1
rc=$?; grep round $O/ub_ab.log; exit $rc
