#!/bin/bash
# gpurun with a wait for a free GPU slot: re-submits ONLY when gpurun reports that nothing ran ("transient":
# no box / slot free, nothing charged); any call that ran — passed, failed or timed out — is final.
#   tools/gpurun_retry.sh <timeout_s> '<command>'  (output of the last attempt on stdout)
T=${1:?timeout}; shift
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpurun_retry] attempt $attempt: no slot ($st); waiting" >&2
  sleep 120
done
exit 3
