#!/bin/bash
# Round-4 evidence run on one GPU: the GPU suite, then optional steps.
#   scripts/gpu_r04.sh TAG [tests] [ab "CFG1" "CFG2" ...] [bench] [dist] [smoke]
# Every GPU step has its own time limit; the first failing step ends the run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04}
shift
mkdir -p $O
while [ $# -gt 0 ]; do
  case "$1" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
      rc=$?; grep -E "passed|failed|FAIL|ERROR" $O/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc ;;
    ab)
      shift; cfgs=()
      while [ $# -gt 0 ] && [[ "$1" == *=* ]]; do cfgs+=("$1"); shift; done
      timeout -k 10 600 python -u scripts/ab_c3.py "${cfgs[@]}" --rounds 4 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
      tail -12 $O/ab.log; continue ;;
    abspmm)
      shift; cfgs=()
      while [ $# -gt 0 ] && [[ "$1" == *=* ]]; do cfgs+=("$1"); shift; done
      timeout -k 10 600 python -u scripts/ab_c3.py "${cfgs[@]}" --spmm-only --rounds 3 > $O/abspmm.log 2>&1 || { tail -20 $O/abspmm.log; exit 1; }
      tail -12 $O/abspmm.log; continue ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_ms'])" ;;
    dist)
      timeout -k 10 300 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_dist_halo.json 2> $O/bench_dist_halo.err || { tail $O/bench_dist_halo.err; exit 1; }
      timeout -k 10 300 python bench.py --dist --exchange allgather --steps 10 --warmup 2 --no-cpu-baseline --spmm-reps 2 > $O/bench_dist_ag.json 2> $O/bench_dist_ag.err || { tail $O/bench_dist_ag.err; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
  shift
done
