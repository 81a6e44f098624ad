#!/bin/bash
# Round 5: C5 library A/Bs (non-temporal stream loads):
#   bash scripts/gpu_r05o.sh TAG lib1 lib2 ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/${1:-r05o}
AB_SCRIPT=ab_c5.py bash scripts/gpu_lib_ab.sh ${1:-r05o}/ab "--steps 10" ${@:2} || exit 1
