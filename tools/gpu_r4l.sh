# round 4: host-side step overheads (DeviceParallel, summed-gather upconv phases, cached flat-source check):
# generator / training GPU tests, the bench, the gap attribution
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_loop.py tests/test_gpu_zopt.py tests/test_gpu_parity.py tests/test_gpu_state.py > gpurun_out/r4l_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4l_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gap_attrib.py --steps 2 --out gpurun_out/r4l_gap.txt > gpurun_out/r4l_gap.log 2>&1
