#!/bin/bash
# Run GPU steps in sequence on the gpurun box; each step has its own time limit; the script stops
# at the first step that faults / aborts / times out (exit >= 124), test failures (rc 1) continue.
#   bash scripts/gpu_run.sh "name1:timeout1:cmd1" "name2:timeout2:cmd2" ...
set -u
mkdir -p gpurun_out
: > gpurun_out/summary.txt
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"
  to="${rest%%:*}"; cmd="${rest#*:}"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc t=$(( $(date +%s) - start ))s" | tee -a gpurun_out/summary.txt
  if [ "$rc" -ge 124 ]; then
    echo "STOP after $name (rc=$rc)" | tee -a gpurun_out/summary.txt
    exit "$rc"
  fi
done
exit 0
