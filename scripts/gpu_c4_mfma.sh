#!/bin/bash
# (1) counter inventory (MFMA names), (2) one PMC pass of MFMA counters on the C3
# bench command, (3) the single-GPU C4 bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-c4mfma}
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || echo "list-avail rc=$?"
grep -o '\bSQ_[A-Z0-9_]*MFMA[A-Z0-9_]*\|\bSQ_INSTS_VALU_[A-Z0-9_]*F64[A-Z0-9_]*' $O/avail.txt | sort -u > $O/mfma_names.txt
cat $O/mfma_names.txt
G=""
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE; do
  grep -qw "$c" $O/avail.txt && G="$G $c"
done
echo "pmc group:$G"
C3ONLY="--no-cpu-baseline --c2-steps 0 --rand-steps 0 --steps 5 --warmup 1 --spmm-reps 2 --c5-steps 3"
timeout -k 10 300 rocprofv3 --pmc $G --output-format csv -d $O/mfma -o p -- python3 $R/bench.py $C3ONLY > $O/mfma.log 2>&1 || { echo "mfma pass rc=$?"; tail -5 $O/mfma.log; exit 1; }
cd $R
timeout -k 10 900 python bench.py --config c4 --steps 10 --warmup 2 --spmm-reps 5 > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
cat $O/c4.json
