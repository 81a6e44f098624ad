#!/bin/bash
# Plan-kernel / Gram-overlap kernel trace, then the SpMM PMC groups (normal vs all-L2 diag).
#   bash scripts/gpu_r04t.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r04t}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_plan -o run -- python3 $R/scripts/plan_trace.py > $O/trace_plan.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/trace_plan.log; exit 1; }
cd $R
bash scripts/pmc_cmd.sh spmm_norm k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_norm.txt 2>&1 || { echo "pmc norm failed"; tail -5 $O/pmc_norm.txt; exit 1; }
LZ_SPMM_DIAG=64 bash scripts/pmc_cmd.sh spmm_diag k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_diag.txt 2>&1 || { echo "pmc diag failed"; tail -5 $O/pmc_diag.txt; exit 1; }
echo done
