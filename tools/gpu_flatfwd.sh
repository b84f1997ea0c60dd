# the training GPU tests on the flat-parameter forward, then a same-box A/B of C3 (ESR_FLAT_FWD 0 / 1, order 0 1 0 1)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/flatfwd.log
: > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_loop.py tests/test_gpu_grid.py tests/test_gpu_ddp.py tests/test_gpu_state.py tests/test_gpu_disc.py -x -q --timeout 300 --timeout-method thread >> $out 2>&1 || exit $?
for v in 0 1 0 1; do
  echo "== ESR_FLAT_FWD=$v" >> $out
  ESR_FLAT_FWD=$v timeout -k 10 200 python3 bench_train.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
done
