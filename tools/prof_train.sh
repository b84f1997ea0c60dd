#!/bin/bash
# rocprofv3 kernel trace of bench_train.py (config 3) -> OUTDIR/trace; summarise with tools/trace_window.py
out=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/trace -o run -- python3 $R/bench_train.py --steps 3 --warmup 2 "$@" > $R/$out/trace.log 2>&1
