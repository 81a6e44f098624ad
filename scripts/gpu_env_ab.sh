#!/bin/bash
# Alternating bench runs under env settings: bash scripts/gpu_env_ab.sh "A=1 B=2" "A=0" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/eab
mkdir -p $O
for round in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --spmm-reps 0 --c2-steps 0 --c5-steps 0 --rand-steps 0 > $O/b_${i}_$round.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/b_${i}_$round.json'));print('[$cfg]', d['value'], d['extra']['kernel_ms_per_step'])"
  done
done
