#!/bin/bash
# Round 6: the k_wf16 drift since round 3 -- the round-3, -4 and -5 libraries
# (built from git history into lib/r03, lib/r04, lib/r05) against the current
# one in alternating processes on one box, C3, 20-step solves, the post-call
# state pass off where a build has it (round 3's has none).
cd "$GRAFT_REPO_ROOT" || exit 1
export AB_FS=0
bash scripts/gpu_lib_ab.sh ${1:-r06c} "--steps 20" r03 r04 r05 cur
