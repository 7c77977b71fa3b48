#!/bin/bash
# Local wrapper (build container side) around gpurun: clears stale step logs, runs the command,
# prints the verdict; re-submits only when gpurun reports an infrastructure-transient failure in which
# nothing ran (status "transient"/rc 3), at most 10 attempts.  Never retries a failing GPU step.
# Usage: bash tools/gpu.sh <timeout-s> '<command>'
lim=$1; shift
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  rm -f gpurun_out/*.log gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > gpurun_out/gpurun_client.txt 2>&1
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d.get('status'))" 2>/dev/null)
  echo "[gpu.sh] attempt $attempt: gpurun rc=$rc status=$st"
  if [ "$st" = "transient" ] || [ $rc -eq 3 ] || grep -q "backing off" gpurun_out/gpurun_client.txt; then
    sleep 75; continue
  fi
  tail -3 gpurun_out/gpurun_client.txt
  exit $rc
done
exit 99
