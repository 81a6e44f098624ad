#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/small_bench.py > gpurun_out/small.json 2> gpurun_out/small.err || exit $?
cat gpurun_out/small.json
