#!/bin/bash
# Local helper: run one gpurun call; if the infrastructure did not run it (transient / box not ready / no slot),
# wait and try again (at most 4 attempts).  A call that ran (whatever its exit status) is never repeated.
# usage: tools/gr.sh TIMEOUT 'command'
t=$1; shift
for a in 1 2 3 4; do
  out=$(timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  echo "$out" | grep -v 'every call sends' | tail -4
  if echo "$out" | grep -q 'status=transient\|stopped responding while being prepared\|backing off\|no box\|no slot'; then
    sleep 45; continue
  fi
  exit $rc
done
exit 3
