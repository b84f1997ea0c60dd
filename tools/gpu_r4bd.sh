# round 4: esr_axpby_gs on the row-walking kernel (bitwise the same): its variant test, training / grid / Z tests,
# same-box A/B of the config-3 step (ESR_AXPBY_ROWS 0 vs 1, ablation library)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_grid.py tests/test_gpu_zopt.py > gpurun_out/r4bd_tests.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_AXPBY_ROWS 0 1
