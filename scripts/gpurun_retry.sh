#!/bin/bash
# Submit one gpurun call and resubmit it ONLY while the pool reports that no box / slot was free
# (exit code 3 or a "transient" verdict with nothing run and nothing charged).  A call that ran --
# whatever its outcome -- is never resubmitted.
#   bash scripts/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=${1:?log}; TO=${2:?timeout}; CMD=${3:?command}
for attempt in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$LOG" && grep -q "run 0.0s\|run Nones" "$LOG"; }; then
    echo "[retry] attempt $attempt: no box (rc=$rc); waiting" >> "$LOG.retries"
    sleep 150
    continue
  fi
  echo "[retry] attempt $attempt finished rc=$rc" >> "$LOG.retries"
  exit $rc
done
exit 3
