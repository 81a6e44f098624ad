#!/bin/bash
# Newton-Schulz sqrtm: probe (accuracy / time against the Jacobi route), the GPU
# suite, the C3 A/B; then the plan-kernel trace and the SpMM PMC groups.
#   bash scripts/gpu_r04u.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-r04u}
mkdir -p $O
timeout -k 10 60 ./scripts/gprobe/sqrtm_probe > $O/sqrtm_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -5 $O/sqrtm_probe.log; exit 1; }
cat $O/sqrtm_probe.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u scripts/ab_c3.py "LZ_SQRTM_NS=1" "LZ_SQRTM_NS=0" --rounds 4 --steps 20 > $O/ns_ab.log 2>&1 || { echo "ab failed rc=$?"; tail -5 $O/ns_ab.log; exit 1; }
grep "^round" $O/ns_ab.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_plan -o run -- python3 $R/scripts/plan_trace.py > $O/trace_plan.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/trace_plan.log; exit 1; }
cd $R
bash scripts/pmc_cmd.sh spmm_norm k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_norm.txt 2>&1 || { echo "pmc norm failed"; tail -5 $O/pmc_norm.txt; exit 1; }
LZ_SPMM_DIAG=64 bash scripts/pmc_cmd.sh spmm_diag k_spmm_seg scripts/spmm_one.py 1e7 4096 16 > $O/pmc_diag.txt 2>&1 || { echo "pmc diag failed"; tail -5 $O/pmc_diag.txt; exit 1; }
echo done
