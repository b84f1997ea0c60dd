# BatchNorm forward statistics in one pass: the BN / discriminator GPU tests, then the config-3 step on the ablation
# library with esr_bn_set_onepass 1 (product) / 0 (two passes), order 1 0 1 0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_disc.py tests/test_gpu_grid.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/bn1_tests.log 2>&1 || exit $?
out=gpurun_out/bn1_ab.log
: > $out
export ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so
for k in 1 0 1 0; do
  echo "== bn_set_onepass=$k" >> $out
  timeout -k 10 200 python3 tools/knob_bench.py bn_set_onepass=$k -- bench_train.py --steps 8 2>/dev/null | grep '^{' >> $out || exit $?
done
