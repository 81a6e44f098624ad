#!/bin/bash
# C4 at N = 8 virtual ranks, halo form, overlap on / off, three repetitions (the
# spread of eight ranks sharing one device).
#   bash scripts/gpu_r04_vr.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04vr}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 600 python -X faulthandler -u scripts/vrank_bench.py --ranks 8 --config c4 --exchange halo --overlap both --steps 10 --warmup 2 --out $O/vr_c4_n8_$r.json > $O/vr_c4_n8_$r.log 2>&1 || { tail -30 $O/vr_c4_n8_$r.log; exit 1; }
  python -c "
import json
d = json.load(open('$O/vr_c4_n8_$r.json'))
print($r, [(x['overlap'], x['ms_per_step_all_ranks'], x['parity']['ok']) for x in d['results']])"
done
