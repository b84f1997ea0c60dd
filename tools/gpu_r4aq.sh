# round 4: fused first D conv block, weights staged in LDS: its tests, timing, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_disc.py -k "first_conv" > gpurun_out/r4aq_first.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dfirst_bench.py > gpurun_out/r4aq_dfirst.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4aq_prof -o dfirst -- python3 tools/dfirst_bench.py > gpurun_out/r4aq_prof.log 2>&1 || exit $?
