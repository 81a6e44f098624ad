#!/bin/bash
# usage: pmc_passes2.sh TAG -- <python script args>; TA/TD/TCP/TCC busy+stall passes
R=$GRAFT_REPO_ROOT
TAG=$1; shift; shift
mkdir -p $R/gpurun_out/pmc_$TAG
cd /tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_$TAG/p$i -o p -- python3 "$@" > $R/gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; }
done <<'GROUPS'
GRBM_GUI_ACTIVE TA_BUSY_avr
TA_TA_BUSY_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum
TA_ADDR_STALLED_BY_TD_CYCLES_sum
TD_CYCLES_sum TD_LOAD_WAVEFRONT_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_RDRET_STALL_sum
TCP_RFIFO_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum
TCC_BUSY_avr TCC_TAG_STALL_sum
TCC_IB_STALL_sum TCC_HIT_sum
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM
GROUPS
