# round 4: C2 step with the HR convs fused / unfused, same box (order A B A B), C2 leg only
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4v_fuse_ab.log
: > $out
for v in 1 0 1 0; do
  echo "== ESR_FUSE_HR1=$v" >> $out
  ESR_FUSE_HR1=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --no-cpu-variants 2>&1 | grep '^{' >> $out || exit $?
done
