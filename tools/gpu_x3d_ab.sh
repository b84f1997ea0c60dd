# 8-channel double-buffered N = 32 x3 conv (ablation variant 88) vs the production one-stage kernel (variant 1):
# per-launch A/B at the config-2 (B=32 and the 16-image stream part, 148²), config-3 (96²) and config-5 (172²) shapes,
# then the C2 bench line per variant
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/x3d_ab.log
: > $out
export ESR_AMD_LIB=exp_lib/libesr_exp.so
for shp in "32 148" "16 148" "16 96" "8 172"; do
  set -- $shp
  AB_B=$1 AB_HW=$2 AB_VARIANTS=1,88 AB_ROUNDS=4 timeout -k 10 300 python3 tools/x3_ab.py >> $out 2>&1 || exit $?
done
for v in 1 88 1 88; do
  echo "== C2 x3-kernel $v" >> $out
  timeout -k 10 200 python3 bench.py --no-legs --no-cpu-baseline --no-op-timers --steps 20 --warmup 5 --x3-kernel $v 2>/dev/null | grep '^{' >> $out || exit $?
done
