#!/usr/bin/env bash
# Submit one gpurun call, resubmitting ONLY while gpurun answers 3 ("no box or slot free right
# now": nothing ran, nothing charged), at most TRIES times, WAIT seconds apart.  Any other exit
# code — including a failed GPU step — ends the loop.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
tries=${TRIES:-8}; wait_s=${WAIT:-240}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$log.attempts"
  [ $rc -ne 3 ] && exit $rc
  sleep "$wait_s"
done
exit 3
