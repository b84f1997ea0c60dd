# round 4: D pre-split + window prefetch: GPU tests of the D, C3 A/B, then the full bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_disc.py tests/test_gpu_grid.py tests/test_gpu_train_loop.py > gpurun_out/r4g_tests.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_DCONV_PRESPLIT 0 1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4g_bench.log 2>&1 || exit $?
bash tools/prof_train.sh gpurun_out/r4g_c3prof
