#!/bin/bash
# Submit one gpurun call; if no box or slot was free (exit 3: nothing ran,
# nothing charged), or the box stopped responding while being prepared (the
# command never started, nothing charged), submit the same call again after a
# pause, at most 12 times.
# Any other outcome (success, failure, refusal, time limit) ends it.
#   scripts/gpu_submit.sh OUTFILE TIMEOUT 'command'
out=$1; t=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$out" 2>&1
  rc=$?
  grep -q "stopped responding while being prepared; retry" "$out" && { sleep 60; continue; }
  [ $rc -ne 3 ] && grep -q -v "no free box\|GPU slot(s) on this pod are busy" "$out" && [ $rc -ne 3 ] && exit $rc
  grep -q "nothing was charged\|no free box\|stopped responding while being prepared; retry" "$out" || exit $rc
  sleep 150
done
exit 3
