# C3 step under each discriminator-kernel knob setting of the ablation library (tools/knob_bench.py), one run each,
# the product settings first and last (box drift)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dknob_sweep.log
: > $out
export ESR_AMD_LIB=exp_lib/libesr_exp.so
for k in "dconv_set_halo=1" "dconv_set_halo=0" "dconv_set_halo=2" "dconv_set_occ3=0" "dconv_set_cw16=0" "dconv_set_rows=1" "wgrad_set_kernel=0" "dconv_set_halo=1"; do
  echo "== $k" >> $out
  timeout -k 10 200 python3 tools/knob_bench.py $k -- bench_train.py --steps 8 2>/dev/null | grep '^{' >> $out || exit $?
done
