#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/small_bench.py > gpurun_out/small.json 2> gpurun_out/small.err || exit $?
cat gpurun_out/small.json
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_lanczos.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
