#!/bin/bash
# Round 6: MALL-residency probe of the C5 SpMM (diagnostic build): hot columns
# (degree order) gathered with the default policy, the rest nt / sc1 / sc1 nt.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
export LZ_HIP_LIB=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib/liblz_hip_diag.so
timeout -k 10 500 python -u scripts/hot_probe.py --rounds 3 "LZ_X=0" "LZ_SPMM_HOT=2000000,1" "LZ_SPMM_HOT=2500000,1" "LZ_SPMM_HOT=3000000,1" \
  "LZ_SPMM_HOT=4000000,1" "LZ_SPMM_HOT=2500000,3" "LZ_SPMM_HOT=3000000,3" > $O/hot_probe2.log 2>&1
rc=$?; tail -12 $O/hot_probe2.log; exit $rc
