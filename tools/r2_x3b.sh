set -o pipefail
mkdir -p gpurun_out
ESR_DGRAD_X3=1 ESR_WGRAD_X3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_loop.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/x3b_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/x3b_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/wgrad_ab.py > gpurun_out/wg_ab.log 2>&1 && \
ESR_DGRAD_X3=1 ESR_WGRAD_X3=1 timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/x3b_train.log 2>&1 && \
ESR_WGRAD_X3=1 timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/x3b_train_nod.log 2>&1 && \
ESR_DGRAD_X3=0 ESR_WGRAD_X3=0 timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/x3b_train_f32.log 2>&1
