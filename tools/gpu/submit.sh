#!/bin/bash
# Local helper (build container side): submit one tools/gpu/run.sh pass through gpurun and,
# only while gpurun answers 3 (no box or slot free, or the box lost before the command ran:
# nothing ran, nothing charged),
# submit the SAME pass again after a pause.  Any other outcome -- success, a failed step, a
# refusal -- ends it: a GPU step that failed is never re-run.
#   tools/gpu/submit.sh LOG TIMEOUT TAG STEP...
LOG=$1; TMO=$2; shift 2
cmd="bash tools/gpu/run.sh"
for a in "$@"; do cmd+=" $(printf '%q' "$a")"; done
for attempt in $(seq 1 ${SUBMIT_ATTEMPTS:-8}); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$cmd" > "$LOG" 2>&1
  rc=$?
  echo "exit $rc (attempt $attempt)" >> "$LOG"
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
