# How the x3 conv's per-image time depends on the workgroups per launch at config-3 shapes (96 x 96 LR; 8 column strips
# of 12): B = 8, 16 (config 3: 392 workgroups for 768 slots), 24, 32, 48.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/occ_probe.log
: > $out
for B in 8 16 24 32 48; do
  timeout -k 10 120 python3 tools/x3_width_probe.py $B 96 128 96 >> $out 2>&1 || exit $?
done
for B in 8 16 32; do
  timeout -k 10 120 python3 tools/x3_width_probe.py $B 96 64 96 >> $out 2>&1 || exit $?
done
