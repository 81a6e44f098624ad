#!/bin/bash
# Round 6: C5's hot-column gathers (LZ_C5_HOT): the tests, then the A/B against
# every column gathered alike (LZ_C5_HOT=0), alternating in one process.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "hot_columns or c5_full or f32_b32 or powerlaw" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/ab_c5.py "LZ_C5_HOT=0" "LZ_C5_HOT=1" --rounds 4 > $O/hot_ab.log 2>&1 || { tail -20 $O/hot_ab.log; exit 1; }
grep round $O/hot_ab.log
