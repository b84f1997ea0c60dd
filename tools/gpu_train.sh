# GPU run: training / checkpoint / Z-opt GPU tests, then the config-3 training bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_loop.py tests/test_gpu_train.py tests/test_gpu_checkpoint.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/train_tests.log 2>&1 && \
timeout -k 10 300 python bench_train.py --steps 5 --warmup 2 > gpurun_out/train_bench.log 2>&1
