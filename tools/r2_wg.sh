set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "weight_gradient_kernels or all_parameter_gradients" > gpurun_out/wg_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/wgrad_ab.py > gpurun_out/wg_ab.log 2>&1
