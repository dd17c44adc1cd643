#!/bin/bash
# gpurun with waits while no box is free (exit 3 / transient); any other outcome returns at once.
for i in $(seq 1 ${TRIES:-12}); do
  out=$(timeout 3000 /usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | tail -${TAILN:-40}
  if echo "$out" | grep -q "status=transient"; then echo "[gpuq] no box (try $i), waiting"; sleep 150; continue; fi
  exit $rc
done
exit 3
