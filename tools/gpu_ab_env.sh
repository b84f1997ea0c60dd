# same-box A/B of the config-3 training step over one environment switch: bash tools/gpu_ab_env.sh VAR A B
# (order A B A B; JSON lines into gpurun_out/ab_env_VAR.log).  Kernel switches (ESR_X3_KERNEL, ESR_X3_NSPLIT) act on
# the ablation library only, so both arms run on it (ESR_AMD_LIB=exp_lib/libesr_exp.so, built by `make exp`).
set -o pipefail
var=$1; a=$2; b=$3
mkdir -p gpurun_out
out=gpurun_out/ab_env_$var.log
: > $out
for v in $a $b $a $b; do
  echo "== $var=$v" >> $out
  env ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so $var=$v timeout -k 10 200 python -u bench_train.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
