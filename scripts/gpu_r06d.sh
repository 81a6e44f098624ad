#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 120 python -u scripts/ub_debug.py 20011 > $O/ub_debug.log 2>&1; rc=$?; cat $O/ub_debug.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/ub_debug.py 1000003 > $O/ub_debug_big.log 2>&1; rc=$?; cat $O/ub_debug_big.log | grep -v amdgpu.ids; exit $rc
