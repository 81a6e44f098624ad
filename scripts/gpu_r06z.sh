#!/bin/bash
# Round 6: repeatability -- the GPU suite twice and the default bench three times on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$i.log 2>&1 || { tail -30 $O/pytest_$i.log; exit 1; }
  tail -1 $O/pytest_$i.log
done
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_ms'],d['extra']['plain_spmm']['roofline']['avg_ms'],d['extra']['c5_block32_f32_powerlaw']['iters_per_s'])"
done
