# GPU run: all -m gpu tests, smoke(), the default bench (usage: gpurun -- bash tools/gpu_full.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/full_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/full_bench.log 2>&1
