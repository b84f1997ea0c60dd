# round 4: fused first D conv block, 32-channel backward chunks: tests, discriminator / training / grid tests, config-3 A/B
# then a same-box A/B of the config-3 step (ESR_DFIRST 0 vs 1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_disc.py -k "first_conv" > gpurun_out/r4av_first.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_disc.py tests/test_gpu_train_loop.py tests/test_gpu_grid.py tests/test_gpu_train.py > gpurun_out/r4av_tests.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_DFIRST 0 1
