# same-box A/B of the config-3 training step: discriminator x3 halo tiles with 128-wide N (default) vs 64 only
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_dnb.log
: > $out
for v in 1 0 1 0; do
  echo "== ESR_DCONV_NB128=$v" >> $out
  ESR_DCONV_NB128=$v timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
