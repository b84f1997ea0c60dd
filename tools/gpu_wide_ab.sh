# N = 32 x3 conv in wider tiles at two workgroups per CU (ablation variants 85: 18 columns, 86: 24 columns) vs the
# production 12-column tiles at three per CU (variant 1): per-launch A/B at the config-2 part shape (B=16, 148²) and
# the full shape (B=32), config 3 (B=16, 96²) and config 5 (B=8, 172²); then the C2 bench line per variant
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/wide_ab.log
: > $out
export ESR_AMD_LIB=exp_lib/libesr_exp.so
for shp in "16 148" "32 148" "16 96" "8 172"; do
  set -- $shp
  AB_B=$1 AB_HW=$2 AB_VARIANTS=1,85,86 AB_ROUNDS=4 timeout -k 10 300 python3 tools/x3_ab.py >> $out 2>&1 || exit $?
done
for v in 1 85 86 1 85 86; do
  echo "== C2 x3-kernel $v" >> $out
  timeout -k 10 200 python3 bench.py --no-legs --no-cpu-baseline --no-op-timers --steps 20 --warmup 5 --x3-kernel $v 2>/dev/null | grep '^{' >> $out || exit $?
done
