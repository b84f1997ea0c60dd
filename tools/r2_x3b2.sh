set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_loop.py tests/test_gpu_zopt.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/x3b2_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/x3b2_rc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/wgrad_ab.py --splits-scale 1 > gpurun_out/wg_ab2.log 2>&1 && \
timeout -k 10 200 python -u bench_train.py --steps 3 --warmup 2 > gpurun_out/x3b2_train.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_train2 -o run -- python3 $R/bench_train.py --steps 3 --warmup 2 > $R/gpurun_out/prof_train2.log 2>&1
