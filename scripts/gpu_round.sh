#!/bin/bash
# End-of-milestone GPU evidence: tests, smoke, bench (+CPU baseline), kernel
# trace/stats profile, FETCH/WRITE PMC passes of the bench command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROOT=$PWD
TAG=${1:-r01}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp
# C3 only (no extras): the stress case and C5 also launch k_fused_pp16 / k_spmm_seg
C3ONLY="--no-cpu-baseline --c2-steps 0 --c5-steps 0 --rand-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $ROOT/bench.py $C3ONLY > $O/trace.json 2> $O/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 $ROOT/bench.py $C3ONLY --steps 5 --warmup 1 --spmm-reps 2 > $O/write.log 2>&1 || exit $?
cd $ROOT
NNZ=$(python -c "import json;print(json.load(open('$O/bench.json'))['config']['nnz_per_gpu'])")
python scripts/pmc_traffic.py $O/fetch $O/write k_fused_pp16 10000000 $NNZ 4096 $O/pmc_k_fused_pp16.json
python scripts/pmc_traffic.py $O/fetch $O/write "k_spmm_seg<double, 16, 48, 768, 8, true, 0, 0>" 10000000 $NNZ 4096 $O/pmc_k_spmm_seg.json  # the MODE-0 (tile) kernel, not the long-tile pass
python scripts/pmc_traffic.py $O/fetch $O/write k_fused_update16 10000000 $NNZ 4096 $O/pmc_k_fused_update16.json
