#!/bin/bash
# rocprofv3 passes over the default inference bench (kernel trace + stats, then FETCH_SIZE and WRITE_SIZE PMC passes,
# each its own run), summarised by tools/prof_summary.py.   usage: tools/prof_bench.sh OUTDIR [bench args...]
out=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
args="--no-cpu-baseline --steps 2 --warmup 1 $*"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/trace -o run -- python3 $R/bench.py $args > $R/$out/trace.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$out/pmc_fetch -o run -- python3 $R/bench.py $args > $R/$out/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$out/pmc_write -o run -- python3 $R/bench.py $args > $R/$out/write.log 2>&1 || exit $?
