#!/bin/bash
# Run one GPU step under its own time limit; log its exit status.  A test failure (1) lets the caller continue; a
# fault, abort, segfault or time limit (anything else) ends the whole GPU call.
# usage: tools/gpu_step.sh SECONDS LOGFILE cmd args...
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "rc=$rc: $*" >> gpurun_out/rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
exit 0
