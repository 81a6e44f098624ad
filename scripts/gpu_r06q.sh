#!/bin/bash
# Round 6: whole-row W'' stores through LDS in the b = 32 fp32 DMA passes (UB, E, U):
# the bitwise tests, then the A/B against the 4-B result-layout stores (LZ_UB_DMA=9).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "f32_b32 or final_state or powerlaw" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_UB_DMA=9" "LZ_UB_DMA=1" --rounds 3 > $O/ub_store_ab.log 2>&1 || { tail -20 $O/ub_store_ab.log; exit 1; }
grep round $O/ub_store_ab.log
timeout -k 10 300 python -u scripts/ab_c5.py "LZ_C5_B2=0 LZ_UB_DMA=9" "LZ_C5_B2=0 LZ_UB_DMA=1" --rounds 3 > $O/e_store_ab.log 2>&1 || { tail -20 $O/e_store_ab.log; exit 1; }
grep round $O/e_store_ab.log
