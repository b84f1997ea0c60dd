set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_loop.py tests/test_gpu_zopt.py tests/test_gpu_train.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r2_tests2.log 2>&1
