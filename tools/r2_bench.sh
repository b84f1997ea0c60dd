set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 && \
timeout -k 10 120 python -u -m pytest tests/test_gpu_bench.py -m gpu -q --timeout 110 --timeout-method thread > gpurun_out/r2_bench_test.log 2>&1 && \
bash tools/prof_bench.sh gpurun_out/prof_r2 --no-legs
