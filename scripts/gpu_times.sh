#!/bin/bash
# per-block timeline of the wavefront launch (scripts/wf_times.py).  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-times}
mkdir -p $O
timeout -k 10 300 python -u scripts/wf_times.py > $O/times.log 2>&1 || { tail -20 $O/times.log; exit 1; }
cat $O/times.log
