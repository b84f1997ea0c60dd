# round 4: tiled stride-1 CEM adjoint + block-per-output border: its tests, Z-opt / training tests, the C5 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cem_adjoint.py tests/test_gpu_zopt.py tests/test_gpu_train.py tests/test_gpu_grid.py -k "not c3" > gpurun_out/r4z_tests.log 2>&1 || exit $?
bash tools/prof_zopt.sh gpurun_out/r4z_c5prof
