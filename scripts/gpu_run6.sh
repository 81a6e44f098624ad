#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab.jsonl
for r in 1 2 4; do
  for hw in 64 4096; do
    LZ_SPMM_RPG=$r timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 | sed "s/^{/{\"rpg\": $r, /" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
