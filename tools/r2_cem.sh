set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cem_np.py -m gpu -k "cem or x3_ring" -v --timeout 200 --timeout-method thread > gpurun_out/r2_cem_tests.log 2>&1; \
timeout -k 10 120 python tools/cem_ab.py > gpurun_out/r2_cem_ab.log 2>&1
