set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_train_loop.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/lr_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/lr_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 2 > gpurun_out/lr_train.log 2>&1 && \
bash tools/prof_train.sh gpurun_out/prof_train7
