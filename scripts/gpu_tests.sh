#!/bin/bash
# GPU test suite (one pytest process; every test bounded by --timeout).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25; exit $rc
