#!/bin/bash
# Round 6 (diagnostic build): the plain SpMM's all-L2 ceiling on the current
# kernel, and k_wf16 with plain (L2-keeping) V_{j+1} stores (LZ_WF_DBG=128).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
export LZ_HIP_LIB=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib/liblz_hip_diag.so
timeout -k 10 300 python -u scripts/ab_c3.py --spmm-only --rounds 3 "LZ_SPMM_DIAG=0" "LZ_SPMM_DIAG=64" \
  "LZ_SPMM_DIAG=64 LZ_SPMM_DIAG_Y=1" > $O/spmm_l2_diag.log 2>&1 || { tail -20 $O/spmm_l2_diag.log; exit 1; }
grep round $O/spmm_l2_diag.log
AB_FS=0 timeout -k 10 300 python -u scripts/ab_c3.py --rounds 3 --steps 20 "LZ_WF_DBG=0" "LZ_WF_DBG=128" > $O/wf_plain_v_ab.log 2>&1
rc=$?; grep round $O/wf_plain_v_ab.log; exit $rc
