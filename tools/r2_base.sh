set -o pipefail
mkdir -p gpurun_out
tools/gpu_step.sh 900 gpurun_out/r2_base_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2_base_bench.log 2>&1
