#!/bin/bash
# Round-4 distributed evidence on one GPU: N = 1 RCCL rehearsals of both
# exchanges, the C4 per-rank share alone at the full grid and at one virtual
# rank's share of the CUs (LZ_GRID_CAP=32), and C4 at N = 8 virtual ranks.
#   scripts/gpu_r04_dist.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04d}
mkdir -p $O
B="--steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2"
timeout -k 10 300 python bench.py --dist $B > $O/bench_dist_halo.json 2> $O/bench_dist_halo.err || { tail $O/bench_dist_halo.err; exit 1; }
timeout -k 10 300 python bench.py --dist --exchange allgather $B > $O/bench_dist_ag.json 2> $O/bench_dist_ag.err || { tail $O/bench_dist_ag.err; exit 1; }
python -c "
import json
for f in ('bench_dist_halo', 'bench_dist_ag'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['ms_per_step'], d['extra']['step_form'])"
timeout -k 10 300 python bench.py --config c4rank $B > $O/bench_c4rank.json 2> $O/bench_c4rank.err || { tail $O/bench_c4rank.err; exit 1; }
LZ_GRID_CAP=32 timeout -k 10 300 python bench.py --config c4rank $B > $O/bench_c4rank_cap32.json 2> $O/bench_c4rank_cap32.err || { tail $O/bench_c4rank_cap32.err; exit 1; }
python -c "
import json
for f in ('bench_c4rank', 'bench_c4rank_cap32'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac'])"
timeout -k 10 900 python -X faulthandler -u scripts/vrank_bench.py --ranks 8 --config c4 --exchange halo --overlap both --steps 10 --warmup 2 --out $O/vr_c4_n8.json > $O/vr_c4_n8.log 2>&1 || { tail -30 $O/vr_c4_n8.log; exit 1; }
tail -4 $O/vr_c4_n8.log
