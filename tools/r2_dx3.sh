set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_train_loop.py tests/test_gpu_train.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/dx3_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/dx3_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/dx3_train.log 2>&1 && \
ESR_DCONV_PRECISION=f32 timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/dx3_train_f32d.log 2>&1 && \
timeout -k 10 200 python -u tools/wgrad_ab.py --splits-scale 1 > gpurun_out/wg_ab3.log 2>&1
