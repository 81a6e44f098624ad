#!/bin/bash
# Round-6 counter evidence (the round-5 recipe) on the current sources (one rocprofv3 mode per run,
# never --pmc with tracing):
#   trace: kernel trace + stats of the C3 bench command and of the C4 per-rank share
#   fetch/write passes (FETCH_SIZE, WRITE_SIZE) of: C3 (k_wf16, plain SpMM),
#     c4rank (k_wf16 wide shape), C5 (the b = 32 fp32 SpMM), the random-column stress case
#   mfma: MFMA busy / MOPS of C3 and c4rank k_wf16 (the full 20-launch solve)
# Summaries: scripts/pmc_summarise_r06.sh on the merged CSVs (here, after the run).
#   scripts/gpu_prof_r05.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
O=$ROOT/gpurun_out/${1:-r06p}
mkdir -p $O
cd /tmp
C3="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0"
C3P="$C3 --steps 20 --warmup 0 --spmm-reps 2"
C4R="--config c4rank --no-cpu-baseline --steps 20 --warmup 0 --spmm-reps 2"
C5="--no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --c5-steps 3"
RAND="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --steps 1 --warmup 0 --spmm-reps 0 --rand-steps 2"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
run() {  # name timeout rocprof-args -- bench-args
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name ok"
}
(cd $ROOT && timeout -k 10 400 python3 bench.py --config c4rank --no-cpu-baseline > $O/bench_c4rank.json 2> $O/bench_c4rank.err) || { echo "c4rank failed"; tail -5 $O/bench_c4rank.err; exit 1; }
echo "c4rank ok"
run trace_c3 400 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 $ROOT/bench.py $C3
run trace_c4r 300 --kernel-trace --stats --output-format csv -d $O/trace_c4r -o run -- python3 $ROOT/bench.py --config c4rank --no-cpu-baseline
run fetch_c3 300 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o p -- python3 $ROOT/bench.py $C3P
run write_c3 300 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o p -- python3 $ROOT/bench.py $C3P
run mfma_c3 300 --pmc $MF --output-format csv -d $O/mfma_c3 -o p -- python3 $ROOT/bench.py $C3P
run fetch_c4r 300 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c4r -o p -- python3 $ROOT/bench.py $C4R
run write_c4r 300 --pmc WRITE_SIZE --output-format csv -d $O/write_c4r -o p -- python3 $ROOT/bench.py $C4R
run mfma_c4r 300 --pmc $MF --output-format csv -d $O/mfma_c4r -o p -- python3 $ROOT/bench.py $C4R
run fetch_c5 300 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o p -- python3 $ROOT/bench.py $C5
run write_c5 300 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o p -- python3 $ROOT/bench.py $C5
run fetch_rand 300 --pmc FETCH_SIZE --output-format csv -d $O/fetch_rand -o p -- python3 $ROOT/bench.py $RAND
run write_rand 300 --pmc WRITE_SIZE --output-format csv -d $O/write_rand -o p -- python3 $ROOT/bench.py $RAND
cd $ROOT && python3 scripts/trace_gaps.py $O/trace_c3/ > $O/gaps_c3.txt 2>&1
find $O -name "*.csv" -size +40M -print -delete
find $O -name "*kernel_trace.csv" -path "*fetch*" -delete
find $O -name "*kernel_trace.csv" -path "*write*" -delete
find $O -name "*kernel_trace.csv" -path "*mfma*" -delete
du -sh $O
echo done
