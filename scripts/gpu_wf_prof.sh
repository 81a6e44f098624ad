#!/bin/bash
# wavefront step: parity + A/B, kernel trace, FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 mode per run)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
O=$ROOT/gpurun_out/${1:-wfprof}
mkdir -p $O
timeout -k 10 400 python -u scripts/wf_check.py --ab-rounds 3 > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
tail -12 $O/check.log
cd /tmp
export LZ_PASS_WF=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $ROOT/scripts/wf_one.py --steps 6 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 $ROOT/scripts/wf_one.py --steps 4 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 $ROOT/scripts/wf_one.py --steps 4 > $O/write.log 2>&1 || exit $?
find $O -name "*.csv" -size +40M -print -delete
grep -h "k_wf16\|k_sqrtm\|k_alpha\|k_wf_deps\|k_gram\|k_strip\|k_col16" $O/trace/*/*kernel_stats.csv 2>/dev/null | cut -c1-200
echo done
