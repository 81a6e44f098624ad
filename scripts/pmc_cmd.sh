#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) of any python command:
#   bash scripts/pmc_cmd.sh TAG KERNEL_SUBSTRING script.py args...
# (set LZ_* env vars before calling)
R=$GRAFT_REPO_ROOT
TAG=$1; K=$2; S=$3; shift 3
case "$S" in /*) ;; *) S=$R/$S ;; esac  # (the passes run from /tmp)
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- python3 "$S" "$@" > $O/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; exit 1; }
done <<'GROUPS'
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum
TD_LOAD_WAVEFRONT_sum TD_STORE_WAVEFRONT_sum
SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC
GROUPS
cd $R && python scripts/pmc_summary.py $O $K > $O/summary.json && cat $O/summary.json
