#!/bin/bash
# virtual-rank rehearsals at bench scale on the final code: C4 as stated at
# N = 8 (the north star's partition) and C3 weak scaling at N = 4, both
# exchanges, checked against the oracle on the global operator.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-vr}
mkdir -p $O
timeout -k 10 900 python -u scripts/vrank_bench.py --ranks 8 --config c4 --exchange both --steps 10 --warmup 2 --out $O/c4_n8.json > $O/c4_n8.log 2>&1 || { tail -30 $O/c4_n8.log; exit 1; }
tail -5 $O/c4_n8.log
timeout -k 10 600 python -u scripts/vrank_bench.py --ranks 4 --config c3 --exchange both --steps 10 --warmup 2 --out $O/c3_n4.json > $O/c3_n4.log 2>&1 || { tail -30 $O/c3_n4.log; exit 1; }
tail -5 $O/c3_n4.log
