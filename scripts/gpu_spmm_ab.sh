#!/bin/bash
# Alternating A/B of SpMM variants: bash scripts/gpu_spmm_ab.sh "v1 v2 ..." [n] [hw]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VARS=${1:-"default p"}
mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in $VARS; do
    if [ "$v" = default ]; then unset LZ_SPMM_KERNEL; else export LZ_SPMM_KERNEL=$v; fi
    timeout -k 10 120 python scripts/spmm_var.py ${2:-1e7} ${3:-4096} || exit $?
  done
done
