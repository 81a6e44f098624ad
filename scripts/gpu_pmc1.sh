#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp
for cfg in "1e7 4096 16" "1e7 64 16"; do
  set -- $cfg
  tag="hw$2_b$3"
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc/sq_$tag -o sq -- python3 $R/scripts/spmm_one.py $1 $2 $3 > $R/gpurun_out/pmc/sq_$tag.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc/tcc_$tag -o tcc -- python3 $R/scripts/spmm_one.py $1 $2 $3 > $R/gpurun_out/pmc/tcc_$tag.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc/fetch_$tag -o fetch -- python3 $R/scripts/spmm_one.py $1 $2 $3 > $R/gpurun_out/pmc/fetch_$tag.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d $R/gpurun_out/pmc/sq2_$tag -o sq2 -- python3 $R/scripts/spmm_one.py $1 $2 $3 > $R/gpurun_out/pmc/sq2_$tag.log 2>&1 || echo "sq2 pass failed rc=$?"
done
