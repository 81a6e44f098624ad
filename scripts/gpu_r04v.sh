#!/bin/bash
# sqrtm probe (Newton-Schulz cap), GPU suite, SpMM all-L2 diagnostic from the
# operator's middle (timing + counters), NS A/B.
#   bash scripts/gpu_r04v.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r04v}
mkdir -p $O
timeout -k 10 60 ./scripts/gprobe/sqrtm_probe > $O/sqrtm_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -5 $O/sqrtm_probe.log; exit 1; }
head -8 $O/sqrtm_probe.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u scripts/ab_c3.py "LZ_SPMM_DIAG=0" "LZ_SPMM_DIAG=64" "LZ_SPMM_DIAG=64 LZ_SPMM_DIAG_Y=1" --spmm-only --rounds 3 > $O/spmm_diag.log 2>&1 || { echo "diag failed rc=$?"; tail -5 $O/spmm_diag.log; exit 1; }
grep "^round" $O/spmm_diag.log
LZ_SPMM_DIAG=64 bash scripts/pmc_cmd.sh spmm_diagmid k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_diag.txt 2>&1 || { echo "pmc diag failed"; tail -5 $O/pmc_diag.txt; exit 1; }
timeout -k 10 300 python -u scripts/ab_c3.py "LZ_SQRTM_NS=1" "LZ_SQRTM_NS=0" --rounds 4 --steps 20 > $O/ns_ab.log 2>&1 || { echo "ab failed rc=$?"; tail -5 $O/ns_ab.log; exit 1; }
grep "^round" $O/ns_ab.log
timeout -k 10 300 python -u scripts/ab_c2.py "LZ_VL_WF=1" "LZ_VL_WF=0" --rounds 4 > $O/c2_ab.log 2>&1 || { echo "c2 ab failed rc=$?"; tail -5 $O/c2_ab.log; exit 1; }
grep "^round" $O/c2_ab.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_plan -o run -- python3 $R/scripts/plan_trace.py > $O/trace_plan.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/trace_plan.log; exit 1; }
cd $R
echo done
