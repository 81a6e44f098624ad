#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab.jsonl
for v in queue tile stream; do
  for hw in 64 4096; do
    LZ_SPMM_KERNEL=$v timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
for bp in 2 3 5 8; do
  LZ_SPMM_BLOCKS_PER_CU=$bp timeout -k 10 120 python scripts/spmm_ab.py 1e7 4096 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
done
timeout -k 10 400 python scripts/spmm_sweep.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || exit $?
