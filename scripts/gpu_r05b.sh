#!/bin/bash
# Round 5, session 1: the -m gpu suite (the b = 32 Newton-Schulz sqrtm tests
# among them); the one-GPU specialised wavefront launch (GEN = false) against
# the general form (lib/genonly, -DLZ_WF_GEN_ONLY) in alternating processes;
# C5 with the b = 32 Newton-Schulz sqrtm against the Jacobi route in one
# process (LZ_SQRTM_NS); the reference's harnesses; the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-r05b}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash scripts/gpu_lib_ab.sh $T/fs1 "--steps 20" cur genonly || exit 1
AB_SCRIPT=ab_c5.py bash scripts/gpu_lib_ab.sh $T/c5unr "--steps 10" cur unr16 || exit 1
timeout -k 10 400 python -u scripts/ab_c5.py "LZ_SQRTM_NS=1" "LZ_SQRTM_NS=0" --rounds 3 --steps 10 > $O/c5_ns_ab.log 2>&1 || { tail -20 $O/c5_ns_ab.log; exit 1; }
tail -12 $O/c5_ns_ab.log
timeout -k 10 400 python -u scripts/ref_harness.py > $O/ref_harness.json 2> $O/ref_harness.err || { tail -20 $O/ref_harness.err; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
