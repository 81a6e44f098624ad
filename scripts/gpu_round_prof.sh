#!/bin/bash
# End-of-milestone GPU evidence, part 2: rocprofv3 kernel trace/stats of the
# C3 bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes and one MFMA
# counter pass (C3 + C5), summaries into gpurun_out/TAG (copied to profiles/).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
TAG=${1:-r02}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp
# C3 only (no extras): the stress case and C5 also launch k_fused_pp16 / k_spmm_seg
C3ONLY="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $ROOT/bench.py $C3ONLY > $O/trace.json 2> $O/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o p -- python3 $ROOT/bench.py --no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 5 --warmup 1 --spmm-reps 2 --c5-steps 3 > $O/mfma.log 2>&1 || exit $?
echo done
