# tap-row weight gradient + halo kernels: op tests, A/B, loop determinism with and without HIP graphs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py -x -v -s --timeout 200 --timeout-method thread -p no:warnings -k "dconv_ops" > gpurun_out/rows_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kernel_determinism.py x3 > gpurun_out/kdet2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/dconv_ab.py > gpurun_out/rows_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/loop_determinism.py f32:f32 > gpurun_out/det4.log 2>&1 || exit $?
ESR_TRAIN_GRAPHS=0 timeout -k 10 300 python -u tools/loop_determinism.py f32:f32 >> gpurun_out/det4.log 2>&1
