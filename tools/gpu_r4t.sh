# round 4: fused HR_conv0 + HR_conv1 (x3 inference): generator parity tests, then the bench and its rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_zopt.py -k "not ring" > gpurun_out/r4t_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4t_bench.log 2>&1 || exit $?
