# same-box A/B of the config-3 training step: LDS-DMA x3 weight gradient (wgrad3d) on / off, order A B A B
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_wgrad.log
: > $out
for v in 1 0 1 0; do
  echo "== ESR_WGRAD3_DMA=$v" >> $out
  ESR_WGRAD3_DMA=$v timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
