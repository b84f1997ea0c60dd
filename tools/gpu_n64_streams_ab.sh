# Under the two-stream forward each N = 64 launch covers 16 images, where the tile-round rule picks 12-column tiles
# (at 32 images it picks 16-column ones): ablation library, --x3-kernel 1 (production rule) vs 64 (N = 64 always
# 16-column), S = 2 and S = 1, order-balanced, no per-launch timers
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/n64_streams_ab.log
: > $out
for v in "2 1" "2 64" "1 1" "1 64" "2 1" "2 64"; do
  set -- $v
  echo "== ESR_STREAMS=$1 x3-kernel $2" >> $out
  ESR_AMD_LIB=exp_lib/libesr_exp.so ESR_STREAMS=$1 timeout -k 10 200 python3 bench.py --no-legs --no-cpu-baseline --no-op-timers --steps 20 --warmup 5 --x3-kernel $2 2>/dev/null | grep '^{' >> $out || exit $?
done
