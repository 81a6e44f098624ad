#!/bin/bash
# rocprofv3 kernel trace + stats of the C3 bench command (the roofline
# kernel's time), then the inter-kernel gaps.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
O=$ROOT/gpurun_out/${1:-trace}
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $ROOT/bench.py --no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0 > $O/trace.json 2> $O/trace.err || exit $?
cd $ROOT && python3 scripts/trace_gaps.py $O/trace | tee $O/gaps.txt
find $O -name "*.csv" -size +40M -print -delete
