# Config-2 step with the second stream's part started later by a spin kernel (ESR_STREAM_DELAY GPU cycles), so that
# the two parts' launches are out of phase; no delay first and last (box drift).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/delay_ab.log
: > $out
for d in 0 50000 100000 150000 200000 300000 0; do
  echo "== $d" >> $out
  ESR_STREAM_DELAY=$d timeout -k 10 300 python3 bench.py --no-legs --steps 20 --warmup 5 --no-op-timers --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit $?
done
