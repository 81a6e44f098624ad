#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for v in b2 b2z b2s b2g; do
  for hw in 64 4096; do
    LZ_SPMM_KERNEL=$v timeout -k 10 120 python scripts/spmm_ab.py 1e7 $hw 16 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
  done
done
cat gpurun_out/ab.jsonl
