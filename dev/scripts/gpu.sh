#!/bin/bash
# gpurun with a retry when the box could not be prepared (status=transient / exit 3: nothing ran,
# nothing charged).  A command that ran and failed is never retried.
#   bash dev/scripts/gpu.sh TIMEOUT 'command'
to=$1; shift
for attempt in 1 2 3; do
  rm -f gpurun_out/summary.txt
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" /tmp/gpurun_last.log; then
    echo "[gpu.sh] box not available (attempt $attempt), waiting" >&2
    sleep 60
    continue
  fi
  tail -3 /tmp/gpurun_last.log
  exit $rc
done
tail -3 /tmp/gpurun_last.log
exit 3
