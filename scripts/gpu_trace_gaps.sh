#!/bin/bash
# kernel timeline of a C3 solve, wavefront step (rocprofv3 kernel trace):
# per-kernel durations and the gaps between consecutive kernels.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-gaps}
mkdir -p $O
for e in 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$e -o run -- python3 scripts/ab_c3.py "LZ_PASS_WF=1" --rounds 2 --steps 20 > $O/tr$e.log 2>&1 || { tail -20 $O/tr$e.log; exit 1; }
done
python3 scripts/trace_gaps.py $O/tr0 | tee $O/gaps.txt
