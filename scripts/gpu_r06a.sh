#!/bin/bash
# Round 6: the CU-partitioned SpMM A/B at C3 and the C5 pass-UB DMA A/B
# (alternating, one process each), plus the round's new GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r06b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_lanczos.py -k "ub_dma_bitwise or final_state" tests/test_gpu_vranks.py::test_vranks_setup_failure_votes \
  > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_UB_DMA=0" "LZ_UB_DMA=1" --rounds 3 > $O/ub_ab.log 2>&1 || { tail -30 $O/ub_ab.log; exit 1; }
tail -12 $O/ub_ab.log
timeout -k 10 300 python -u scripts/ab_c3.py --spmm-only --rounds 2 \
  "LZ_SPMM_PF=0" "LZ_SPMM_PF=2,8,96" "LZ_SPMM_PF=1,8,96" "LZ_SPMM_PF=2,8,32" "LZ_SPMM_PF=2,16,192" > $O/pf_ab.log 2>&1
rc=$?; tail -30 $O/pf_ab.log; exit $rc
