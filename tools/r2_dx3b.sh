set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/dx3b_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/dx3b_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/dconv_ab.py > gpurun_out/dconv_ab.log 2>&1 && \
timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/dx3b_train.log 2>&1
