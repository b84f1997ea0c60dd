#!/bin/bash
# rocprofv3 kernel trace of bench_zopt.py (config 5) -> OUTDIR/trace; summarise with tools/trace_window.py / trace_gaps.py
out=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/trace -o run -- python3 $R/bench_zopt.py --steps 4 --warmup 4 "$@" > $R/$out/trace.log 2>&1
