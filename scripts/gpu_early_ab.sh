#!/bin/bash
# Early sqrtm: the wavefront tests, an in-process A/B at C3 (early on / off /
# off on the early form's grid), then the default bench.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-early}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanczos.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "wavefront or b16 or c3_full or sqrtm or golden" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_c3.py "LZ_WF_EARLY=0" "LZ_WF_EARLY=1" "LZ_WF_EARLY=0 LZ_WF_GRID=255" --rounds 5 --steps 20 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -30 $O/ab.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
