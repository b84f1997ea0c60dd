# GPU run: rocprofv3 kernel trace of the default bench (extra bench args in $ARGS) -> gpurun_out/tb/trace
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/tb
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tb/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-legs --steps 2 --warmup 1 $ARGS > $R/gpurun_out/tb/trace.log 2>&1
