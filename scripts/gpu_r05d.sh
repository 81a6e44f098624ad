#!/bin/bash
# Round 5: the stream-ordered workspace fills against the run-to-run
# differences of the distributed b = 32 fp32 solve (before: ~45 % of runs at N = 1).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05d
for N in 1 2; do
timeout -k 10 300 python -u scripts/flake_ag_step0.py 60 1 $N > gpurun_out/r05d/fix_n$N.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/r05d/fix_n$N.log; exit 1; }
tail -1 gpurun_out/r05d/fix_n$N.log
done
timeout -k 10 400 python -u scripts/flake_b32_ag.py 12 allgather "LZ_SQRTM_NS=1" "LZ_SQRTM_NS=0" > gpurun_out/r05d/fix_ag.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/r05d/fix_ag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05d/fix_ag.log | tail -2
timeout -k 10 400 python -u scripts/flake_b32_ag.py 12 halo "LZ_SQRTM_NS=1" "LZ_SQRTM_NS=0" > gpurun_out/r05d/fix_halo.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/r05d/fix_halo.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05d/fix_halo.log | tail -2
