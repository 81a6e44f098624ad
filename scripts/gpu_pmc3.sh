#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/pmc_passes2.sh buf_hw4096 -- $GRAFT_REPO_ROOT/scripts/spmm_one.py 1e7 4096 16
python scripts/pmc_summary.py gpurun_out/pmc_buf_hw4096 k_spmm_buf
