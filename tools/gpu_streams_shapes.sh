# Multi-stream forward A/B at the C3 / C5 generator shapes (inference forward only, no timers): does splitting the
# batch over S streams pay where one launch under-fills the 768 workgroup slots (3 per CU)?
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/streams_shapes.log
: > $out
run() {  # label, S, args...
  local label=$1 s=$2; shift 2
  echo "== $label S=$s" >> $out
  ESR_STREAMS=$s timeout -k 10 200 python3 bench.py --no-legs --no-cpu-baseline --no-op-timers --steps 20 --warmup 5 "$@" 2>/dev/null | grep '^{' >> $out || exit $?
}
for s in 1 2 3 1 2 3; do run c5_172 $s --variant latent --batch 8 --lr-size 152; done
for s in 1 2 3 1 2 3; do run c3_96 $s --no-cem --batch 16 --lr-size 96; done
for s in 1 2 1 2; do run c5l_154 $s --variant latent --batch 8 --lr-size 134; done
