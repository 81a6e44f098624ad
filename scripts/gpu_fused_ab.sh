#!/bin/bash
# Fused pass-1 variants: GPU Lanczos tests under each, then alternating bench runs.
#   bash scripts/gpu_fused_ab.sh "default s"
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VARS=${1:-"default s"}
O=gpurun_out/fab
mkdir -p $O
for v in $VARS; do
  [ "$v" = default ] && unset LZ_FUSED_KERNEL || export LZ_FUSED_KERNEL=$v
  timeout -k 10 300 python -m pytest tests/test_gpu_lanczos.py tests/test_gpu_dist.py -x -q -p no:cacheprovider > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/t_$v.log)"
done
for round in 1 2; do
  for v in $VARS; do
    [ "$v" = default ] && unset LZ_FUSED_KERNEL || export LZ_FUSED_KERNEL=$v
    timeout -k 10 200 python bench.py --no-cpu-baseline --spmm-reps 0 > $O/b_${v}_$round.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/b_${v}_$round.json'));print('$v', d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['extra']['kernel_ms_per_step'])"
  done
done
