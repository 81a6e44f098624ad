#!/bin/bash
# C4 on the final code: the whole 40M-row operator on one GPU (parity against
# the oracle on the 1e9-nonzero operator) and the 8-rank decomposition as
# virtual ranks on one device (halo form, overlap on and off).
#   bash scripts/gpu_r04_c4.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04c4}
mkdir -p $O
timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4_1gpu.json 2> $O/bench_c4_1gpu.err || { tail $O/bench_c4_1gpu.err; exit 1; }
cut -c1-300 $O/bench_c4_1gpu.json
timeout -k 10 900 python -X faulthandler -u scripts/vrank_bench.py --ranks 8 --config c4 --exchange halo --overlap both --steps 10 --warmup 2 --out $O/vr_c4_n8.json > $O/vr_c4_n8.log 2>&1 || { tail -30 $O/vr_c4_n8.log; exit 1; }
tail -3 $O/vr_c4_n8.log | cut -c1-300
