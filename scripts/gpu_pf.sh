#!/bin/bash
# A/B of the fused pass-1 kernels: parity tests under the candidate, then bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CAND=${1:-p}
LZ_FUSED_KERNEL=$CAND timeout -k 10 600 python -m pytest tests/test_gpu_lanczos.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_$CAND.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$CAND.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in $CAND ws; do
LZ_FUSED_KERNEL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --spmm-reps 0 > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['extra']['kernel_ms_per_step'])"
done
