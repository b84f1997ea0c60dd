# round 4: N = 64 12-column tiles in the product dispatch: conv parity tests, training / Z tests, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_zopt.py tests/test_gpu_grid.py > gpurun_out/r4al_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4al_bench.log 2>&1 || exit $?
