# same-box A/B of the C3 training step: weight gradients on a second stream (ESR_WGRAD_STREAM) and the x3 trunk-level
# data gradients (ESR_TRUNK_X3), order-balanced A B A B; then a C5 iteration twice
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_stream.log
: > $out
for v in 1 0 1 0; do
  echo "== ESR_WGRAD_STREAM=$v" >> $out
  ESR_WGRAD_STREAM=$v timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
for v in 0 1; do
  echo "== ESR_TRUNK_X3=$v (WGRAD_STREAM=0)" >> $out
  ESR_WGRAD_STREAM=0 ESR_TRUNK_X3=$v timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
for r in 1 2; do
  echo "== C5 run $r" >> $out
  timeout -k 10 200 python -u bench_zopt.py --steps 5 --warmup 2 2>&1 | grep '^{' >> $out || exit $?
done
