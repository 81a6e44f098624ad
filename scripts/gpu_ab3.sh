#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k spmm > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_m.log; if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab.jsonl
for v in buf tile; do
  for hw in 64 4096; do
    LZ_SPMM_KERNEL=$v timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
cat gpurun_out/ab.jsonl
