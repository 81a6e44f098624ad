#!/bin/bash
# TCP/TA counters of the gather probes (one --pmc pass per group)
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcprobe; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d $O/a -o p -- $R/scripts/gprobe/split_probe > $O/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- $R/scripts/gprobe/split_probe > $O/b.log 2>&1 || exit 1
echo ok
