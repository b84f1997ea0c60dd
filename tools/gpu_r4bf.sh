# round 4: the input adjoint's four corner outputs on a block per corner: Z / training / grid tests, the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zopt.py tests/test_gpu_grid.py tests/test_gpu_train.py tests/test_gpu_validation.py > gpurun_out/r4bf_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4bf_bench.log 2>&1 || exit $?
