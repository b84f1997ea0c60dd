# same-box A/B of the config-3 training step (LEG train, default) or the config-5 Z iteration (LEG zopt) over one
# environment switch: bash tools/gpu_ab_env.sh VAR A B [LEG] (order A B A B; JSON lines into
# gpurun_out/ab_env_VAR[_LEG].log).  Kernel switches that only the ablation library reads
# (ESR_X3_KERNEL, ESR_X3_NSPLIT, ESR_AXPBY_ROWS, ESR_WGRAD3D_UNROLL: esr_amd/_lib.py) run both arms on it; every other (Python-level)
# switch runs both arms on the product library, the code that ships.
set -o pipefail
var=$1; a=$2; b=$3; leg=${4:-train}
mkdir -p gpurun_out
out=gpurun_out/ab_env_$var${4:+_$4}.log
: > $out
case $var in
  ESR_X3_KERNEL|ESR_X3_NSPLIT|ESR_AXPBY_ROWS|ESR_WGRAD3D_UNROLL) lib="ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so" ;;
  *) lib="" ;;
esac
for v in $a $b $a $b; do
  echo "== $var=$v ${lib:+(ablation library)}" >> $out
  env $lib $var=$v timeout -k 10 200 python -u bench_$leg.py --steps 5 --warmup 4 2>&1 | grep '^{' >> $out || exit $?
done
