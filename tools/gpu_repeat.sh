# Same-box repeatability of the three headline measurements at HEAD: the C2 line (bench.py --no-legs, 20 steps) three
# times, the C3 step (bench_train.py) and the C5 iteration (bench_zopt.py) twice each.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/repeat.log
: > $out
for i in 1 2 3; do
  echo "== C2 $i" >> $out
  timeout -k 10 300 python3 bench.py --no-legs --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | grep '^{' >> $out || exit $?
done
for i in 1 2; do
  echo "== C3 $i" >> $out
  timeout -k 10 300 python3 bench_train.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
  echo "== C5 $i" >> $out
  timeout -k 10 300 python3 bench_zopt.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
done
