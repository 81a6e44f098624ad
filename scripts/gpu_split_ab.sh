#!/bin/bash
# CU split of the wavefront step (LZ_WF_SPLIT): parity under the split, then an
# in-process A/B at C3.  Usage: scripts/gpu_split_ab.sh TAG "cfg" "cfg" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-split}; shift
mkdir -p $O
LZ_WF_SPLIT=${SPLIT_CHECK:-20} timeout -k 10 300 python -u scripts/wf_check.py --ab-rounds 0 > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
tail -8 $O/check.log
timeout -k 10 400 python -u scripts/ab_c3.py "$@" --rounds 3 --steps 10 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
