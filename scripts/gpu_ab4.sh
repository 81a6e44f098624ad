#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in w0 w1 w2; do
LZ_SPMM_KERNEL=$v timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k spmm > gpurun_out/pytest_$v.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$v.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
: > gpurun_out/ab.jsonl
for v in buf w0 w1 w2; do
  for hw in 64 4096; do
    LZ_SPMM_KERNEL=$v timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
cat gpurun_out/ab.jsonl
