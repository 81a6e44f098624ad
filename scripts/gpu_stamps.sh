#!/bin/bash
# sqrtm-block stamps (scripts/wf_stamps.py), then the early A/B.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps}
mkdir -p $O
timeout -k 10 300 python -u scripts/wf_stamps.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
