#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench command
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ROOT=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $ROOT/gpurun_out/prof/bench.json 2> $ROOT/gpurun_out/prof/bench.err || exit $?
cd $ROOT && find gpurun_out/prof -name "*stats*" && cat gpurun_out/prof/bench.json
