#!/bin/bash
# Alternating A/B of pass-1 variants (bench lines, no CPU baseline), 3 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
for v in ${@:-ws q0 r}; do
LZ_FUSED_KERNEL=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --spmm-reps 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$r $v',d['value'],d['extra']['kernel_ms_per_step']['fused_spmm_pass'])"
done
done
