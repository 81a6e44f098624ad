#!/bin/bash
# Round-3 counter evidence (one rocprofv3 mode per run, never --pmc with tracing):
#   trace   kernel trace + stats of the C3 bench command (roofline kernel time)
#   fetch / write      FETCH_SIZE, WRITE_SIZE passes of the C3 command (pass 1, pass 2, plain SpMM)
#   rfetch / rwrite    the same on the random-column stress operator (its k_spmm_seg only)
#   mfma    MFMA busy / MOPS counters of C3 and C5
# Summaries are made from the merged CSVs (scripts/pmc_traffic.py, pmc_mfma.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
TAG=${1:-r03}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp
C3ONLY="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0"
RAND="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 2 --steps 1 --warmup 0 --spmm-reps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $ROOT/bench.py $C3ONLY > $O/trace.json 2> $O/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/rfetch -o p -- python3 $ROOT/bench.py $RAND > $O/rfetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/rwrite -o p -- python3 $ROOT/bench.py $RAND > $O/rwrite.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o p -- python3 $ROOT/bench.py --no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 5 --warmup 1 --spmm-reps 2 --c5-steps 3 > $O/mfma.log 2>&1 || exit $?
# keep only the CSVs the summaries need (the merge back is capped)
find $O -name "*.csv" -size +40M -print -delete
du -sh $O
echo done
