# split-precision halo discriminator kernels: op tests vs float64, determinism (kernels, D step), A/B, loop margins
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py -x -v -s --timeout 200 --timeout-method thread -p no:warnings -k "dconv_ops" > gpurun_out/x6_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_loop.py -x -v -s --timeout 200 --timeout-method thread -p no:warnings -k "deferred" > gpurun_out/redo_test.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kernel_determinism.py f32 > gpurun_out/kdet.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kernel_determinism.py x6 >> gpurun_out/kdet.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/d_determinism.py > gpurun_out/ddet.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/dconv_ab.py > gpurun_out/x6_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/loop_margin.py x3:x6 f32:x6 > gpurun_out/x6_margins.log 2>&1
