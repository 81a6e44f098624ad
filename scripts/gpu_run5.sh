#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_lanczos.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab.jsonl
for v in tile queue; do
  for hw in 64 4096; do
    LZ_SPMM_KERNEL=$v timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
LZ_SPMM_KERNEL=tile timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
