set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zopt.py tests/test_gpu_train.py tests/test_gpu_train_loop.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/zx3_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/zx3_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench_zopt.py > gpurun_out/zx3_zopt.log 2>&1 && \
ESR_DGRAD_X3=0 timeout -k 10 200 python -u bench_zopt.py > gpurun_out/zx3_zopt_f32.log 2>&1
