#!/bin/bash
# Library A/B on one GPU: builds of liblz_hip.so (lib/<name>/liblz_hip.so, or
# "cur" for lib/liblz_hip.so) in alternating processes, 3 rounds.
#   scripts/gpu_lib_ab.sh TAG "ab_c3.py arguments" name1 name2 ...
# (AB_SCRIPT=ab_c5.py: the C5 harness instead)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-libab}
ARGS=$2
shift 2
mkdir -p $O
L=$PWD/gpu-implementation-of-signle-and-block-lanczos_amd/lib
for i in 1 2 3; do
  line="round $i:"
  for nm in "$@"; do
    if [ "$nm" = cur ]; then lib=$L/liblz_hip.so; else lib=$L/$nm/liblz_hip.so; fi
    LZ_HIP_LIB=$lib timeout -k 10 200 python -u scripts/${AB_SCRIPT:-ab_c3.py} LZ_SPMM_TOUCH=0 $ARGS --rounds 1 > $O/${nm}_$i.log 2>&1 || { tail $O/${nm}_$i.log; exit 1; }
    line="$line  $nm [$(grep '^round 0' $O/${nm}_$i.log | sed 's/round 0 \[LZ_SPMM_TOUCH=0\]//')]"
  done
  echo "$line"
done
