# round 4: batched weight-gradient reductions (esr_wgrad_reduce_multi): training tests, loop margins, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_loop.py tests/test_gpu_grid.py > gpurun_out/r4am_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4am_bench.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/loop_margin.py x3:x3 f32:f32 > gpurun_out/r4am_loop_margins.txt 2>&1 || exit $?
