#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool reports that NOTHING ran (no free
# box / slot, or the box was taken away before the command started: status=transient, exit 3 --
# nothing charged, no GPU step executed).  A call whose command ran is never re-submitted.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None charged=0.0s" "$LOG"; then
    echo "[gpurun_when_free] attempt $attempt: nothing ran ($(grep -o 'status=[a-z]*' "$LOG" | tail -1)); waiting" >> "$LOG.retries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
