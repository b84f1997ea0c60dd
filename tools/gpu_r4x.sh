# round 4: tiled stride-1 CEM adjoint: its tests, the Z-opt / training tests that run it, the C5 and C3 legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cem_adjoint.py tests/test_gpu_zopt.py tests/test_gpu_train.py tests/test_gpu_grid.py -k "not c3" > gpurun_out/r4x_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4x_bench.log 2>&1 || exit $?
