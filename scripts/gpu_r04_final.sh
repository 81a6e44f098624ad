#!/bin/bash
# Round-4 closing evidence: the stress case's SpMM counters (FETCH / WRITE on the
# current lz_spmm.hip), then the default bench line.
#   bash scripts/gpu_r04_final.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
O=$ROOT/gpurun_out/${1:-r04f2}
mkdir -p $O
cd /tmp
RAND="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --rand-steps 2"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/${c}_rand -o p -- python3 $ROOT/bench.py $RAND > $O/${c}_rand.log 2>&1 || { echo "$c pass failed rc=$?"; tail -5 $O/${c}_rand.log; exit 1; }
  echo "$c ok"
done
find $O -name "*kernel_trace.csv" -delete
cd $ROOT
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
echo done
