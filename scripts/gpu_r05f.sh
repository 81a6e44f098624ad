#!/bin/bash
# Round 5: counters of the column-panel SpMM candidate and of k_spmm_seg at C3
# (one rocprofv3 --pmc pass per group, never with tracing).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05f
mkdir -p $O
cd /tmp
for which in panel seg; do
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/${which}_p$i -o p -- python3 $R/scripts/panel_ab.py --which $which --rounds 1 --reps 2 > $O/${which}_p$i.log 2>&1 || { echo "$which pass $i ($grp) failed rc=$?"; tail -3 $O/${which}_p$i.log; exit 1; }
done <<'GROUPS'
SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum
FETCH_SIZE
WRITE_SIZE
GROUPS
echo "$which ok"
done
cd $R
for which in panel seg; do
  mkdir -p $O/$which; for d in $O/${which}_p*; do [ -d "$d" ] && mv $d $O/$which/; done
done
python scripts/pmc_summary.py $O/panel k_spmm_panel > $O/panel.json && python scripts/pmc_summary.py $O/seg "k_spmm_seg<double, 16, 48, 768, false, 0" > $O/seg.json
cat $O/panel.json $O/seg.json
find $O -name "*kernel_trace.csv" -delete
