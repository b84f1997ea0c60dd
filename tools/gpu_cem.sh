# GPU run: the CEM stencil parity tests and tools/cem_ab.py timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "cem" > gpurun_out/cem_test.log 2>&1 && \
timeout -k 10 120 python tools/cem_ab.py > gpurun_out/cem_ab.log 2>&1
