set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_loop.py tests/test_gpu_train.py tests/test_gpu_checkpoint.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/adam_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/adam_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 2 > gpurun_out/adam_train.log 2>&1 && \
ESR_ADAM_FUSED=0 timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 2 > gpurun_out/adam_train_off.log 2>&1
