#!/bin/bash
# Round-4 session: SpMM PMC groups (normal vs all-L2 diag) and the per-solve
# overhead A/B (beta_0 Gram beside the plans, final-state grid, final state off).
#   bash scripts/gpu_r04s.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wf_plan.py \
  > $O/wf_plan_tests.log 2>&1 || { echo "wf_plan tests failed rc=$?"; tail -30 $O/wf_plan_tests.log; exit 1; }
tail -2 $O/wf_plan_tests.log
timeout -k 10 400 python -u scripts/ab_c3.py "AB_FS=1" "LZ_GRAM_SIDE=0 LZ_WF_DEPS4=0" "LZ_FS_BPC=0" "LZ_FS_BPC=6" "AB_FS=0" \
  --rounds 4 --steps 20 > $O/fs_ab.log 2>&1 || { echo "fs_ab failed rc=$?"; tail -5 $O/fs_ab.log; exit 1; }
tail -30 $O/fs_ab.log
bash scripts/pmc_cmd.sh spmm_norm k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_norm.txt 2>&1 || { echo "pmc norm failed"; tail -5 $O/pmc_norm.txt; exit 1; }
LZ_SPMM_DIAG=64 bash scripts/pmc_cmd.sh spmm_diag k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_diag.txt 2>&1 || { echo "pmc diag failed"; tail -5 $O/pmc_diag.txt; exit 1; }
echo done
