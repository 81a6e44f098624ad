#!/bin/bash
# Round 5: C5's long-tile pass beside the tile pass (the list step 0 queued) --
# the C5 tests on that build, then the library A/B on the C5 step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
L=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib
LZ_HIP_LIB=$L/conc/liblz_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lanczos.py tests/test_gpu_vranks.py -m gpu -x -v -k "c5_full_size or final_state or powerlaw or b32 or fused_any_b" --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_conc.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest_conc.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest_conc.log | head; tail -30 $O/pytest_conc.log; exit $rc; }
AB_SCRIPT=ab_c5.py bash scripts/gpu_lib_ab.sh r05n/ab "--steps 10" cur conc || exit 1
