#!/bin/bash
# Round 6: the pass-E form's DMA staging A/B (C5 operator), and the counters of
# the plain SpMM as it runs against the same kernel on a masked stream of 7/8
# of the CUs (diagnostic build; one --pmc pass per group, scripts/pmc_cmd.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_C5_B2=0 LZ_UB_DMA=0" "LZ_C5_B2=0 LZ_UB_DMA=1" --rounds 3 > $O/e_dma_ab.log 2>&1 || { tail -20 $O/e_dma_ab.log; exit 1; }
grep round $O/e_dma_ab.log
export LZ_HIP_LIB=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib/liblz_hip_diag.so
timeout -k 10 500 bash scripts/pmc_cmd.sh r06n_spmm_all "k_spmm_seg<double, 16, 48, 768, false, 0, false, false, false>" scripts/ab_c3.py --spmm-only --rounds 1 "LZ_SPMM_PF=0" > $O/pmc_all.log 2>&1 || { tail -5 $O/pmc_all.log; exit 1; }
timeout -k 10 500 bash scripts/pmc_cmd.sh r06n_spmm_masked "k_spmm_seg<double, 16, 48, 768, false, 0, false, false, true>" scripts/ab_c3.py --spmm-only --rounds 1 "LZ_SPMM_PF=1,0" > $O/pmc_masked.log 2>&1
rc=$?; tail -3 $O/pmc_masked.log; exit $rc
