#!/bin/bash
# SpMM A/B on one GPU: the previous build (lib/head) against the current one in
# alternating processes, then in-process knobs of the current build.
#   scripts/gpu_spmm_ab.sh TAG "CFG1" "CFG2" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-spmmab}
shift
mkdir -p $O
HEAD=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib/head/liblz_hip.so
for i in 1 2 3; do
  LZ_HIP_LIB=$HEAD timeout -k 10 200 python -u scripts/ab_c3.py LZ_SPMM_TOUCH=0 --spmm-only --rounds 2 > $O/head_$i.log 2>&1 || { tail $O/head_$i.log; exit 1; }
  timeout -k 10 200 python -u scripts/ab_c3.py LZ_SPMM_TOUCH=0 --spmm-only --rounds 2 > $O/new_$i.log 2>&1 || { tail $O/new_$i.log; exit 1; }
  echo "head $(grep -o 'spmm [0-9.]* ms' $O/head_$i.log | tail -1)   new $(grep -o 'spmm [0-9.]* ms' $O/new_$i.log | tail -1)"
done
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u scripts/ab_c3.py "$@" --spmm-only --rounds 3 > $O/knobs.log 2>&1 || { tail -20 $O/knobs.log; exit 1; }
  tail -16 $O/knobs.log
fi
