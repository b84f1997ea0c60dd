# round 4: input adjoint per pixel, vectorised grad amax / lrelu backward: training + Z tests, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cem_adjoint.py tests/test_gpu_zopt.py tests/test_gpu_train.py tests/test_gpu_train_loop.py tests/test_gpu_grid.py tests/test_gpu_zobj.py > gpurun_out/r4aa_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4aa_bench.log 2>&1 || exit $?
