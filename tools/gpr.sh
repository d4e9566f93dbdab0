#!/bin/bash
# gpurun with retries while the pool has no box free (exit 3 / transient
# status): at most 6 tries, 60 s apart. usage: bash tools/gpr.sh <timeout> '<command>'
T=$1
shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null; then exit $rc; fi
  echo "[gpr] try $i: no box (rc=$rc), retrying in 60 s"
  sleep 60
done
exit 3
