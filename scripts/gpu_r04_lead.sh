#!/bin/bash
# Pacing lead of the wide wavefront shape at C4's per-rank share (n = 5M, 25 per
# row, half width 65,536; lmin = 28 positions, default lmin + 3).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04lead}
mkdir -p $O
timeout -k 10 900 python -u scripts/ab_c3.py --n 5000000 --nnz-per-row 25 --halfwidth 65536 --steps 10 --rounds 3 \
  "LZ_WF_LEAD=31" "LZ_WF_LEAD=28" "LZ_WF_LEAD=29" "LZ_WF_LEAD=34" "LZ_WF_LEAD=38" "LZ_WF_LEAD=44" > $O/lead_ab.log 2>&1 || { echo "ab failed rc=$?"; tail -5 $O/lead_ab.log; exit 1; }
grep "^round" $O/lead_ab.log
