#!/bin/bash
# Round 6: STREAM-style HBM ceilings for the passes' access mixes (scripts/gprobe/stream_probe.hip).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 120 scripts/gprobe/stream_probe > $O/stream_probe.log 2>&1; rc=$?
cat $O/stream_probe.log; exit $rc
