# round 4: native im2col / col2im for the D's first conv, BN running buffers in the BN launch: D / training tests, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_disc.py tests/test_gpu_train_loop.py tests/test_gpu_grid.py tests/test_gpu_state.py tests/test_gpu_validation.py > gpurun_out/r4ai_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4ai_bench.log 2>&1 || exit $?
