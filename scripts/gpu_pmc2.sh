#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export LZ_SPMM_KERNEL=tile
bash scripts/pmc_passes.sh tile_hw4096 -- $GRAFT_REPO_ROOT/scripts/spmm_ab.py 1e7 4096 16
bash scripts/pmc_passes.sh tile_hw64 -- $GRAFT_REPO_ROOT/scripts/spmm_ab.py 1e7 64 16
