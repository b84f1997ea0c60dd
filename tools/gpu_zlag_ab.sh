# Z-optimisation: overflow flags read one iteration later (ESR_ZOPT_LAG=1, default) vs right after each iteration;
# same box, order-balanced; then the Z-opt GPU tests (overflow redo, parity)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/zlag_ab.log
: > $out
for v in 0 1 0 1; do
  echo "== ESR_ZOPT_LAG=$v" >> $out
  ESR_ZOPT_LAG=$v timeout -k 10 200 python3 bench_zopt.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_zopt.py tests/test_gpu_zobj.py tests/test_gpu_grid.py -x -q --timeout 300 --timeout-method thread -k "zopt or zobj or c5 or Z or z_" >> $out 2>&1 || exit $?
