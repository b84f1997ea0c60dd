# Config-2 step under uneven two-stream batch splits (ESR_STREAM_SPLIT), product library with the narrow column tile
# off (the parent commit's library, exp_lib/libesr_head.so), equal split first and last (box drift).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/split_ab.log
: > $out
export ESR_AMD_LIB=$PWD/exp_lib/libesr_head.so
for sp in 16,16 18,14 20,12 22,10 24,8 14,18 16,16; do
  echo "== $sp" >> $out
  ESR_STREAM_SPLIT=$sp timeout -k 10 300 python3 bench.py --no-legs --steps 20 --warmup 5 --no-op-timers --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit $?
done
for sp in "11,11,10" "12,12,8" "14,10,8"; do
  echo "== S3 $sp" >> $out
  ESR_STREAMS=3 ESR_STREAM_SPLIT=$sp timeout -k 10 300 python3 bench.py --no-legs --steps 20 --warmup 5 --no-op-timers --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit $?
done
