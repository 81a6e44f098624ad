cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/fnz
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "fixed_nnz or spmm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fnz/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|ERROR" gpurun_out/fnz/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_c3.py "LZ_SPMM_FNZ=0" "LZ_SPMM_FNZ=1" --spmm-only --rounds 5 > gpurun_out/fnz/ab.log 2>&1
rc=$?; tail -12 gpurun_out/fnz/ab.log; exit $rc
