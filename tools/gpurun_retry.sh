#!/bin/bash
# Re-submit a gpurun call only when the box never started the command (status=transient,
# i.e. "the GPU box stopped responding while being prepared"); any run that started is
# reported as is, success or failure.
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[retry] transient box failure, attempt $i" >&2
    sleep 90
    continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"
exit $rc
