# round 4: fused first D conv block timing (fused vs general) + rocprof kernel stats of that micro-benchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dfirst_bench.py > gpurun_out/r4ap_dfirst.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4ap_prof -o dfirst -- python3 tools/dfirst_bench.py > gpurun_out/r4ap_prof.log 2>&1 || exit $?
