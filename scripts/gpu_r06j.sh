#!/bin/bash
# Round 6: the plain SpMM on a CU-masked stream with every CU enabled (the
# masked queue's own cost), then the k_wf16 drift A/B (round-3/4/5 libraries).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 200 python -u scripts/ab_c3.py --spmm-only --rounds 2 "LZ_SPMM_PF=0" "LZ_SPMM_PF=0,0" "LZ_SPMM_PF=1,0" \
  > $O/pf_mask_ab.log 2>&1 || { tail -20 $O/pf_mask_ab.log; exit 1; }
grep round $O/pf_mask_ab.log
timeout -k 10 900 bash scripts/gpu_r06c.sh r06j_drift
