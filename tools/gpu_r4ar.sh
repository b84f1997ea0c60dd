# round 4: fused first D conv block (LDS weights in the backward): tests, timing, config-3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_disc.py -k "first_conv" > gpurun_out/r4ar_first.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dfirst_bench.py > gpurun_out/r4ar_dfirst.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_DFIRST 0 1
