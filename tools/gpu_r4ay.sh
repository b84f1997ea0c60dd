# round 4: weight-gradient reduce with batched loads (bitwise the same sums): training tests, config-3 kernel view
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_grid.py tests/test_gpu_disc.py > gpurun_out/r4ay_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/torch_prof_train.py --device > gpurun_out/r4ay_torchdev.log 2>&1 || exit $?
timeout -k 10 300 python -u bench_train.py > gpurun_out/r4ay_c3.log 2>&1 || exit $?
