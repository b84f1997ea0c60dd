# round 4: HR_conv1's data gradient on esr_dfirst_fwd_padded: training / grid / Z / validation tests, config-3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_grid.py tests/test_gpu_zopt.py tests/test_gpu_validation.py tests/test_gpu_train_loop.py > gpurun_out/r4bh_tests.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_HR1_DFIRST 0 1
