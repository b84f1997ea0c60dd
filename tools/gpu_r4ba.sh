# round 4: the RRDB gradient max fused into the previous RRDB's closing add on a row-walking kernel (one atomic per
# block; bitwise the same scale): training / grid / disc / Z tests, kernel view, A/B of the fusion
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_grid.py tests/test_gpu_disc.py tests/test_gpu_zopt.py > gpurun_out/r4ba_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/torch_prof_train.py --device > gpurun_out/r4ba_torchdev.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_AMAX_FUSED 0 1
