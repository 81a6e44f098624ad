#!/bin/bash
# Round-5 GPU evidence: the -m gpu suite (one process, every test bounded),
# then the default bench line.
#   bash scripts/gpu_r05.sh TAG [pytest args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r05a}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|ERROR" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
