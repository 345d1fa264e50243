#!/bin/bash
# Submit one gpurun call; when gpurun reports that NOTHING ran (exit 3: no box
# or slot free, box lost while being prepared -- nothing charged), submit the
# same call again after a pause, at most MAX_TRIES (default 6) times.  Any other exit (the command
# ran, passed or failed) ends it: a failing GPU run is never repeated.
# usage: tools/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for attempt in $(seq 1 ${MAX_TRIES:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -eq 3 ] || break
  echo "attempt $attempt: no box (rc 3), waiting" >> "$log.tries"
  sleep 120
done
echo "rc=$rc" >> "$log"
exit $rc
