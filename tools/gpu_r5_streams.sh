# Round 5 multi-stream lease: the S A/B (tools/gpu_streams_ab.sh), then the bench line with union-of-intervals timing
# at S=1 and S=2 (--no-legs), then the rocprof pass of the default (S=2) bench.
set -o pipefail
bash tools/gpu_streams_ab.sh r5s || exit $?
for s in 1 2; do
  ESR_STREAMS=$s timeout -k 10 300 python3 bench.py --no-legs --steps 20 --warmup 5 > gpurun_out/r5s_bench_s$s.log 2>&1 || exit $?
done
bash tools/gpu_verify.sh r5s c2prof
